"""Times the copy forms of tools/copy_probe.hip (built into raincast_gnn/_native/var/copy_probe/)
over 1 GiB and 4 GiB buffers, plus torch's copy_; prints read+write TB/s per form."""
import ctypes
import os
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "raincast-gnn_amd", "raincast_gnn", "_native", "var",
                               "copy_probe", "copy_probe.so"))
lib.copy_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_void_p]
NAMES = ["block256x8 nt/nt", "block256x8", "block256x8 nt-store", "block512x4", "block256x4",
         "block256x16", "stride2048x256x4", "stride8192x256x8", "block1024x4"]
dev = torch.device("cuda:0")
for gib in (1, 4):
    nbytes = gib << 30
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream(dev)
    def timed(fn, reps=10):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        return 2 * nbytes / (e0.elapsed_time(e1) * 1e-3 / reps) / 1e12
    for m, name in enumerate(NAMES):
        tb = timed(lambda: lib.copy_probe(m, src.data_ptr(), dst.data_ptr(), nbytes, st.cuda_stream))
        ok = torch.equal(dst[:4096], src[:4096]) and torch.equal(dst[-4096:], src[-4096:])
        print(f"{gib} GiB  {name:22s} {tb:6.2f} TB/s  {'ok' if ok else 'WRONG'}", flush=True)
    print(f"{gib} GiB  torch copy_              {timed(lambda: dst.copy_(src)):6.2f} TB/s", flush=True)
    del src, dst
    torch.cuda.empty_cache()
