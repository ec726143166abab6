# A/B per-layer timing of every build under v2e2v_amd/variants/ (one process per build)
for f in v2e2v_amd/variants/*.so; do
  CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py ${1:-64} >> gpurun_out/layers.jsonl 2>> gpurun_out/layers.err || exit 1
done
