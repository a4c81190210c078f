mkdir -p gpurun_out/r04s
for rep in 1 2; do
  for v in new hp2 h0 h0p2; do
    if [ $v = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_$v.so; fi
    timeout -k 10 200 python -u tools/e2e_sweep.py --pageable-only --sizes 4096,8192,16384,32768 --grid "" --out gpurun_out/r04s/sweep_${v}_$rep.json > gpurun_out/r04s/sweep_${v}_$rep.log 2>&1 || exit 1
  done
done
