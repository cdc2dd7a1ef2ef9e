#!/bin/bash
# Round 4: which header candidates a strict stage at 3 waves/SIMD loses (diagnostic)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_DUMP_CANDS=gpurun_out/cands_sw4.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > gpurun_out/cd4.log 2>&1 || { tail -20 gpurun_out/cd4.log; exit 1; }
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_sw3.so NDFL_DUMP_CANDS=gpurun_out/cands_sw3.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > gpurun_out/cd3.log 2>&1 || { tail -20 gpurun_out/cd3.log; exit 1; }
python3 - <<'PY'
import numpy as np
a=np.fromfile('gpurun_out/cands_sw4.bin',dtype=np.uint64); b=np.fromfile('gpurun_out/cands_sw3.bin',dtype=np.uint64)
sa,sb=set(a.tolist()),set(b.tolist())
lost=sorted(sa-sb); extra=sorted(sb-sa)
print('sw4',len(a),'sw3',len(b),'lost',len(lost),'extra',len(extra))
seg=np.array(lost,dtype=np.uint64)//(65536*8)
print('lost first', lost[:10]); print('lost seg', seg[:10].tolist())
segs_all=a//(65536*8); import collections
cnt=collections.Counter(segs_all.tolist())
print('cands per seg of lost segs', [cnt[int(x)] for x in seg[:20]])
d=np.diff(np.array(lost,dtype=np.int64)); print('lost spacing (first 20)', d[:20].tolist())
print('lost mod 32 hist', collections.Counter([int(x)%32 for x in lost]).most_common(8))
PY
