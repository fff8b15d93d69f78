set -u
cd $GRAFT_REPO_ROOT
bash tools/sweep.sh tools/sweep_r1a.txt > gpurun_out/sweep_out.txt 2>&1; rc=$?; echo "sweep rc=$rc"; [ $rc -gt 5 ] && exit $rc
bash tools/pmc.sh tools/pmc_final.txt > gpurun_out/pmc_out.txt 2>&1; rc=$?; echo "pmc rc=$rc"
exit $rc
