set -o pipefail
ROOT=$PWD
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-frames 0 > gpurun_out/bench.log 2>&1 || exit 1
KFX_LIB_PATH=$PWD/slam-kinectfusion_amd/lib/var_raytrace/libkfx.so timeout -k 10 200 python3 tools/ray_trace.py 30 > gpurun_out/rt30.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $ROOT/gpurun_out/pmcr/p1 -- python3 $ROOT/bench.py --steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0 > $ROOT/gpurun_out/pmcr_p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $ROOT/gpurun_out/pmcr/p2 -- python3 $ROOT/bench.py --steps 20 --warmup 5 --profile-frames 2 --cpu-frames 0 > $ROOT/gpurun_out/pmcr_p2.log 2>&1 || exit 1
