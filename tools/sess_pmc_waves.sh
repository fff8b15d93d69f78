cd $GRAFT_REPO_ROOT
bash tools/sweep.sh tools/sweep_r1f.txt > gpurun_out/sweep_out.txt 2>&1 || exit $?
bash tools/pmc.sh tools/pmc_final.txt > gpurun_out/pmc_out.txt 2>&1
