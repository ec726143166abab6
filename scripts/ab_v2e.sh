cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in base flog noleak; do
  CISTA_HIP_LIB=v2e2v_amd/variants/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abv_$v -o run -- python3 scripts/v2e_prof.py 4 > gpurun_out/abv_$v.out 2>&1 || exit $?
done
echo done
