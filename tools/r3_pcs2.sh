# helper-cache diagnostics (lone wave, open loop), then PC sampling of the ensemble headline kernel
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_LIB=$PWD/primesim_amd/libprimeuncore_c4prof.so timeout -k 10 200 python tools/prof_regions.py -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/r3c_regions_single_open.txt 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > /tmp/pcs_list.txt 2>&1; grep -i -B2 -A12 "pc_sampl\|PC Sampling" /tmp/pcs_list.txt | head -80 > gpurun_out/r3c_pcs_list.txt
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 4194304 --output-format csv -d /tmp/pcs_st -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu --no-extras > gpurun_out/r3c_pcs_st.log 2>&1
rc=$?; echo "stochastic rc=$rc" >> gpurun_out/r3c_pcs_st.log
if [ $rc -eq 0 ]; then python tools/pcs_summary.py /tmp/pcs_st "" gpurun_out/r3c_pcs_st_summary.txt 400; ls -laR /tmp/pcs_st | head -30 >> gpurun_out/r3c_pcs_st.log; exit 0; fi
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d /tmp/pcs_ht -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu --no-extras > gpurun_out/r3c_pcs_ht.log 2>&1
rc=$?; echo "host_trap rc=$rc" >> gpurun_out/r3c_pcs_ht.log
if [ $rc -eq 0 ]; then python tools/pcs_summary.py /tmp/pcs_ht "" gpurun_out/r3c_pcs_ht_summary.txt 400; ls -laR /tmp/pcs_ht | head -30 >> gpurun_out/r3c_pcs_ht.log; fi
exit 0
