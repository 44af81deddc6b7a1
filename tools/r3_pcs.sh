# PC sampling of one simulation alone on the GPU (latency mode), plus the M/G/1 fuzz
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -k 10 180 python -u -m pytest tests/test_gpu_mg1.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_mg1_fuzz.log 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d gpurun_out/pcs/st -o run -- python bench.py --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/pcs/st.log 2>&1
rc=$?
echo "stochastic rc=$rc" >> gpurun_out/pcs/st.log
if [ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d gpurun_out/pcs/ht -o run -- python bench.py --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/pcs/ht.log 2>&1
  echo "host_trap rc=$?" >> gpurun_out/pcs/ht.log
fi
exit 0
