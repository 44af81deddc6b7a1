# Final measurements of the shipped build: GPU suite, smoke, PMC fabric traffic (same build), the driver's
# bench config carrying that traffic, rocprofv3 kernel stats of the same command.  tools/r3_final.sh TAG
T=${1:-r3r}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 400 python tools/pmc_traffic.py --work /tmp/pmc --out gpurun_out/${T}_traffic.json -- --steps 5 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_traffic.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traffic-json gpurun_out/${T}_traffic.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras --traffic-json gpurun_out/${T}_traffic.json > gpurun_out/${T}_bench_under_rocprof.json 2> gpurun_out/${T}_rocprof.log || exit 1
cp /tmp/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
du -sh gpurun_out
