"""tt_search_topk (serving top-k) through the C ABI, both the fused scan (Q <= 64) and
the GEMM + column-split path, against an exact reference: integer-valued operands make
every dot product exact in fp32 whatever the summation order, so rankings -- including
ties, which must go to the lower document index -- are compared bit-exactly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, dtype_code  # noqa: E402

DEV = "cuda"


def ref_topk(q, d, k):
    s = (q.double() @ d.double().t()).cpu()
    out_i, out_v = [], []
    for row in s:
        order = sorted(range(row.shape[0]), key=lambda j: (-float(row[j]), j))[:k]
        out_i.append(order)
        out_v.append([float(row[j]) for j in order])
    return torch.tensor(out_i), torch.tensor(out_v)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Q,N,h,k", [(1, 3000, 64, 3), (5, 1025, 128, 1), (64, 4100, 32, 16), (9, 777, 512, 5),
                                     (70, 9000, 64, 3), (130, 5000, 96, 16)])
def test_search_topk_exact(dt, Q, N, h, k):
    g = torch.Generator().manual_seed(Q * 1000 + N)
    q = torch.randint(-3, 4, (Q, h), generator=g).float()
    d = torch.randint(-3, 4, (N, h), generator=g).float()
    d[N // 2] = d[N // 3]            # exact ties: the lower index must rank first
    d[N - 1] = d[7]
    lib = _lib.load()
    qd, dd = q.to(DEV), d.to(DEV, dt)
    idx = torch.empty(Q, k, dtype=torch.int32, device=DEV)
    val = torch.empty(Q, k, dtype=torch.float32, device=DEV)
    ws = torch.empty(max(lib.tt_search_ws_size(dtype_code(dt), Q, N, h, k), 1), dtype=torch.uint8, device=DEV)
    call("tt_search_topk", dtype_code(dt), qd.data_ptr(), Q, dd.data_ptr(), N, h, k, idx.data_ptr(), val.data_ptr(),
         ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    ri, rv = ref_topk(q, d, k)
    assert torch.equal(idx.cpu().long(), ri)
    assert torch.equal(val.cpu().double(), rv.double())


def test_search_topk_rejects_bad_args():
    lib = _lib.load()
    q = torch.zeros(1, 12, device=DEV)
    d = torch.zeros(4, 12, device=DEV)
    out = torch.empty(1, 8, dtype=torch.int32, device=DEV)
    with pytest.raises(_lib.TTError, match="multiple of 8"):
        call("tt_search_topk", 0, q.data_ptr(), 1, d.data_ptr(), 4, 12, 1, out.data_ptr(), None, None,
             torch.cuda.current_stream().cuda_stream)
    q = torch.zeros(1, 16, device=DEV)
    d = torch.zeros(4, 16, device=DEV)
    with pytest.raises(_lib.TTError, match="k=5"):
        call("tt_search_topk", 0, q.data_ptr(), 1, d.data_ptr(), 4, 16, 5, out.data_ptr(), None, None,
             torch.cuda.current_stream().cuda_stream)
    del lib
