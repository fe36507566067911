cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_mlp_hmc.py f32 6 > gpurun_out/probe_mlp_hmc_r05.log 2>&1 &&
timeout -k 10 300 python -u tools/probe_mlp_hmc.py f64 6 >> gpurun_out/probe_mlp_hmc_r05.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && HMCX_HMC_HOST_LOOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hmc -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_mlp_hmc.py f32 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_hmc.log 2>&1
