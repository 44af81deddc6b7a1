# Round-3 full check of the tree: GPU suite, smoke, the driver's bench config, rocprofv3 kernel stats.
#   tools/r3_full.sh TAG   (outputs under gpurun_out/TAG_*)
T=${1:-r3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_bench_under_rocprof.json 2> gpurun_out/${T}_rocprof.log || exit 1
exit 0
