set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ab
: > gpurun_out/ab/lat.jsonl
for rep in 1 2 3 4; do
  for lib in base product; do
    for F in 20 1; do
      if [ $lib = base ]; then e="VPTMCM_LIB=base"; else e="VPTMCM_X=0"; fi
      out=$(timeout -k 10 120 env $e python3 tools/launch_latency.py --passes $F --regions 40 2>>gpurun_out/ab/err.txt) || exit 1
      echo "{\"lib\": \"$lib\", \"F\": $F, \"r\": $out}" >> gpurun_out/ab/lat.jsonl
    done
  done
done
