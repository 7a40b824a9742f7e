cd $GRAFT_REPO_ROOT
for L in ${WEXP_LIBS:-tree}; do
  if [ $L = tree ]; then E=""; else E="PRT_LIB_DIR=$PWD/$L"; fi
  echo "== $L" >> gpurun_out/w4.log
  timeout -k 10 120 env $E python3 tools/latency.py --scene car_boxed --iters 40 --walk 0.02 default hybrid:hot_pct=45,hot_kernel=coop4 >> gpurun_out/w4.log 2>&1 || exit 1
  timeout -k 10 120 env $E python3 tools/latency.py --scene car_boxed --iters 40 --walk 0.02 --start 24 --hold default >> gpurun_out/w4.log 2>&1 || exit 1
done
