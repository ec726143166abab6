# A/B timing of voxelizer builds under v2e2v_amd/variants/ (960-window call, HIP events)
timeout -k 10 120 python scripts/vox_prof.py 960 10 > gpurun_out/vox_ab.jsonl || exit 1
for f in v2e2v_amd/variants/*.so; do
  echo -n "$(basename $f) " >> gpurun_out/vox_ab.jsonl
  CISTA_HIP_LIB=$f timeout -k 10 120 python scripts/vox_prof.py 960 10 >> gpurun_out/vox_ab.jsonl || exit 1
done
cat gpurun_out/vox_ab.jsonl
