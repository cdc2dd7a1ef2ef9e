#!/bin/bash
# Round 5: header-set parity (finder change), the aligned-emit A/B (parity tests + bench pairs), the
# emit pass's WRITE_SIZE at 4/8/16 waves per CU, the 8-rank one-GPU rehearsal of the driver's
# command, then configurations 1/2/3/5.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_headers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hdr_c.log 2>&1 || { tail -30 gpurun_out/hdr_c.log; exit 1; }
tail -1 gpurun_out/hdr_c.log
NDFL_LIB_PATH=$L/libndfl_ealign.so timeout -k 10 400 python -u -m pytest tests/test_gpu_emit_fast.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ef_align.log 2>&1 || { tail -30 gpurun_out/ef_align.log; exit 1; }
tail -1 gpurun_out/ef_align.log
for k in 1 2; do for lib in libndfl.so libndfl_ealign.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-verify > gpurun_out/bc_$lib$k.log 2>&1 || { tail -20 gpurun_out/bc_$lib$k.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/bc_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
bash scripts/r05/emit_writes.sh || exit 1
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/rehearse8.sh || exit 1
bash scripts/r05/configs.sh || exit 1
