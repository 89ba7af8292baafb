# parity of the default library, then alternating A/B of variants: tools/gpu_try.sh "<variants>" "<c3 variants>"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_regimes.py > gpurun_out/t.log 2>&1; rc=$?
tail -n 3 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh 3 "--steps 20 --warmup 5 --c1-frames 0 --host-frames 0 --c3-frames 0 --c5-frames 0" $1 || exit 1
[ -z "$2" ] || bash tools/ab_bench.sh 1 "--config c3 --steps 20 --warmup 5 --c1-frames 0 --host-frames 0 --profile-frames 2" $2
