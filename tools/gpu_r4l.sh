# Full GPU suite + smoke on this build, then the PMC traffic passes (the column-split
# forward launched plainly under rocprofv3: its cooperative launch crashes rocprofv3's
# process teardown, profiles/r04_rocprof_crash_k.txt)
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4l_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4l_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l_smoke.txt 2>&1 || exit 1
grep smoke gpurun_out/r4l_smoke.txt
TT_GRU_XC_COOP=0 timeout -k 10 900 bash tools/pmc_bench.sh r4l || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/pmc_r4l/summary.json'))
for k,v in d.items():
    if 'hbm_bytes_est' in v and v['hbm_bytes_est']>1e9: print(k[:60], round(v['hbm_bytes_est']/1e9,2), v.get('dispatches'))
"
