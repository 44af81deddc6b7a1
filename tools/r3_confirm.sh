# Confirmation on the final tree: GPU suite, smoke, and bench.py with no flags (its defaults)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3n_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3n_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r3n_bench_default.json 2> gpurun_out/r3n_bench_default.log || exit 1
