# full GPU check at the working tree: all -m gpu tests, then the driver's bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t.log 2>&1; rc=$?
tail -n 3 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err && echo bench ok && tail -c 1500 gpurun_out/b1.json
