cd $GRAFT_REPO_ROOT
PARTS="0 default 524288" bash scripts/ab_parts.sh && \
NDFL_LIB_PATH=$GRAFT_REPO_ROOT/deflate-library-java_amd/lib/libndfl_phase.so NDFL_FIND_PART_BITS=0 NDFL_STATS=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/abparts/phase_dense.log 2>&1 && grep "\[ndfl\] count" gpurun_out/abparts/phase_dense.log | tail -2 && \
NDFL_LIB_PATH=$GRAFT_REPO_ROOT/deflate-library-java_amd/lib/libndfl_phase.so NDFL_STATS=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/abparts/phase_sparse.log 2>&1 && grep "\[ndfl\] count" gpurun_out/abparts/phase_sparse.log | tail -2
