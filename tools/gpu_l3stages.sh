set -o pipefail
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for st in 0 41 42 43 4; do
HMCX_L3_STOP=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_l3_$st -o run --output-format csv -- python3 $R/tools/probe_mlp.py 20 > $R/gpurun_out/prof_l3_$st.log 2>&1 || { tail -5 $R/gpurun_out/prof_l3_$st.log; exit 1; }
grep "k_mm<float, 2" $R/gpurun_out/prof_l3_$st/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/stop=$st /"
done
