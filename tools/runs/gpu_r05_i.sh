# r05 i: VMM adjacent-commit probe
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05i; mkdir -p $O
timeout -k 10 60 $R/tools/ubench/vmm > $O/vmm.log 2>&1; rc=$?; echo "vmm rc=$rc"
grep "mode\|strategy" $O/vmm.log
