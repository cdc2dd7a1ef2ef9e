cd $GRAFT_REPO_ROOT
M=deflate-library-java_amd
for v in base NDFL_EXP_NOCOPY NDFL_EXP_NOWAIT "NDFL_EXP_NOCOPY -DNDFL_EXP_NOWAIT"; do
  if [ "$v" != base ]; then make -C $M clean > /dev/null; make -C $M HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -w -D$v" > /dev/null 2>&1 || exit 1; fi
  echo "== $v"
  NDFL_NOCHECK=1 timeout -k 10 300 python scripts/prof_types.py 268435456 > gpurun_out/exp.log 2>&1 || { tail -5 gpurun_out/exp.log; exit 1; }
  grep ratio gpurun_out/exp.log | awk '{print $1, $6, $7}'
done
