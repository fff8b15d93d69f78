# Tile-swap experiment: bit identity, stamps of a fused launch, ABBA timing sweep (analysis)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_bits.py dump gpurun_out/base.json > gpurun_out/ab.log 2>&1
VPTMCM_LIB=swap timeout -k 10 200 python tools/ab_bits.py dump gpurun_out/swap.json >> gpurun_out/ab.log 2>&1
timeout -k 10 60 python tools/ab_bits.py cmp gpurun_out/base.json gpurun_out/swap.json >> gpurun_out/ab.log 2>&1
VPTMCM_LIB=stampswap timeout -k 10 300 python tools/stamp_profile.py > gpurun_out/stamp_swap.json 2> gpurun_out/stamp.err
timeout -k 10 800 bash tools/sweep.sh tools/sweep_swap.txt
