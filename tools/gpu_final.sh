# round-end check: all GPU tests, the driver's bench line, and the C5 single-GPU record
set -o pipefail
bash tools/gpu_full.sh || exit $?
timeout -k 10 400 python3 bench.py --config c5 --steps 20 --warmup 5 --cpu-frames 0 --c1-frames 0 --c3-frames 0 --c5-frames 0 --host-frames 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
tail -c 600 gpurun_out/c5.json
