# config [2] reference golden through both kernel families (+ every 1944 parity test); MEASURE=1 re-measures bounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c2gold
rm -f gpurun_out/c2gold/sp.jsonl
if [ -n "$MEASURE" ]; then export LDPC_PARITY_MEASURE=1; fi  # re-measure FAILURE_BOUNDS (rule (i) only)
LDPC_PARITY_LOG=$PWD/gpurun_out/c2gold/sp.jsonl timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_soft_parity.py tests/test_gpu_parity.py -k "1944" > gpurun_out/c2gold/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/c2gold/pytest.log; exit $rc
