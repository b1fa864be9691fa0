"""Verify the LDS XOR swizzles of csrc/tt_gemm_core.h are bank-conflict free for the
gfx950 lane groups (MI355X_MICROARCH.md §LDS): ds_read_b128 on the K-contig image,
ds_read_b64_tr_b16 on the K-outer bf16 image, ds_read_b32 on the K-outer fp32 image."""

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]


def kc_off(row, c):
    return row * 128 + 16 * (c ^ ((row >> 1) & 7))


def ko_v(k):
    return (k & 3) | (((k >> 3) & 1) << 2)


def ko16_off(k, c):
    return k * 256 + 16 * (c ^ (ko_v(k) << 1))


def ko32_elem(k, m):
    return k * 512 + 4 * (m ^ (16 * ((k >> 2) & 1)))


def main():
    bad = 0
    for rb in range(0, 256, 16):
        for kk in (0, 1):
            for g in B128_GROUPS:
                slots = {(kc_off(rb + (l & 15), (l >> 4) + 4 * kk) // 16) % 16 for l in g}
                bad += len(slots) != 16
    print("K-contig ds_read_b128 conflicting groups:", bad)
    bad = 0
    for ks in (0, 32):
        for mt in range(8):
            for second in (0, 1):
                for half in (0, 1):
                    slots = set()
                    for l in range(32 * half, 32 * half + 32):
                        g, i = l >> 4, l & 15
                        q, p = i >> 2, i & 3
                        k = ks + 8 * g + q + 4 * second
                        cc = mt * 4 + p
                        slots.add(((ko16_off(k, cc >> 1) + 8 * (cc & 1)) // 8) % 32)
                    bad += len(slots) != 32
    print("K-outer bf16 ds_read_b64_tr_b16 conflicting half-waves:", bad)
    bad = 0
    for ks in (0, 16):
        for mt in range(8):
            for e in range(4):
                for half in (0, 1):
                    banks = set()
                    for l in range(32 * half, 32 * half + 32):
                        k = ks + 4 * (l >> 4) + e
                        banks.add((ko32_elem(k, mt * 16 + (l & 15)) // 4) % 32)
                    bad += len(banks) != 32
    print("K-outer fp32 ds_read_b32 conflicting half-waves:", bad)


if __name__ == "__main__":
    main()
