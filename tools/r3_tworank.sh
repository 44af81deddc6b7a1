# bench.py --gpus 2 launching its own two ranks, both on card 0 (gloo for the reduction)
export TMPDIR=/tmp
mkdir -p gpurun_out
PU_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu --dist-backend gloo > gpurun_out/r3s_two_rank.json 2> gpurun_out/r3s_two_rank.log || exit 1
