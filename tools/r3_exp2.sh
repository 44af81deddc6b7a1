# compile-time-geometry A/B (single replica and ensemble), PC sampling
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -k 10 120 python bench.py --replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras > gpurun_out/r3_b1.log 2>&1 || exit 1
AB_OTHER=c4geo timeout -k 10 200 bash tools/ab_single.sh > gpurun_out/r3_ab_single_c4geo.txt 2>&1 || exit 1
timeout -k 10 400 bash tools/ab_multi.sh 2 main c4geo > gpurun_out/r3_ab_multi_c4geo.txt 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
timeout -k 10 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d gpurun_out/pcs/st -o run -- python bench.py --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/pcs/st.log 2>&1
echo "stochastic rc=$?" >> gpurun_out/pcs/st.log
exit 0
