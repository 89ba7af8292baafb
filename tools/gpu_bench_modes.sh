set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err && echo b1 ok &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --mode slab --icp allreduce --cpu-frames 0 --c1-frames 0 > gpurun_out/b2.json 2> gpurun_out/b2.err && echo b2 ok &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --config c5 --cpu-frames 0 --c1-frames 0 --host-frames 0 > gpurun_out/b3.json 2> gpurun_out/b3.err && echo b3 ok
