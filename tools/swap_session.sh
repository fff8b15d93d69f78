# A/B bit identity of the tile-swap test builds against the product (analysis)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_bits.py dump gpurun_out/base.json > gpurun_out/ab.log 2>&1
for v in ${SWAP_VARIANTS:-swapno swapself swap}; do
  VPTMCM_LIB=$v timeout -k 10 200 python tools/ab_bits.py dump gpurun_out/$v.json >> gpurun_out/ab.log 2>&1
  timeout -k 10 60 python tools/ab_bits.py cmp gpurun_out/base.json gpurun_out/$v.json >> gpurun_out/ab.log 2>&1 || echo "$v differs" >> gpurun_out/ab.log
done
