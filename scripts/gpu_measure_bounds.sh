set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fb
rm -f gpurun_out/fb/g.jsonl
LDPC_PARITY_MEASURE=1 LDPC_PARITY_LOG=$PWD/gpurun_out/fb/g.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fb/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/fb/pytest.log; exit $rc
