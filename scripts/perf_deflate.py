import os, sys, time, torch, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'deflate-library-java_amd/python')); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import ndfl, corpus
ctx = ndfl.Context(0)
L = ndfl._lib.load()
for name, n in [(a.split(":")[0], int(a.split(":")[1]) << 20) for a in (sys.argv[1:] or ["c4:4096", "zeros:1024", "rand:1024"])]:
    if name == "c4": x = corpus.c4_mixed(n, device="cuda")
    elif name == "zeros": x = torch.zeros(n, dtype=torch.uint8, device="cuda")
    else: x = torch.randint(0,256,(n,),dtype=torch.uint8,device="cuda")
    cap = L.ndfl_deflate_bound(n, 65536) + 64
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for it in range(3):
        t = time.time()
        eb, crc = ctx.deflate_chunks_raw(None, 0, 32768, x.data_ptr(), n, 65536, 3, True, 0, out.data_ptr(), cap, 3, crc=0)
        dt = time.time() - t
        print(name, it, "bytes", eb//8, "ratio %.3f" % (eb/8/n), "wall %.2f ms" % (dt*1e3), "kernel %.2f ms" % ctx.last_kernel_ms(),
              "GB/s(N+C) %.1f" % ((n + eb/8)/ctx.last_kernel_ms()/1e6), flush=True)
    del x, out
