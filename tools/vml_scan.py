import ctypes, os, sys, time
import numpy as np
import torch
L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
MODE = ctypes.c_longlong(0x140102)
name = sys.argv[1]
f = getattr(L, name)
f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong]
def vml(x):
    out = np.empty_like(x); f(len(x), x.ctypes.data, out.ctypes.data, MODE); return out
ref64 = {"vmsAcos": np.arccos, "vmsSqrt": np.sqrt, "vmsSin": np.sin, "vmsCos": np.cos}[name]
lo_bits, hi_bits = int(sys.argv[2], 16), int(sys.argv[3], 16)
CH = 1 << 24
tot = mism = 0
fr_mis, fr_ok_near = [], []
t0 = time.time()
for start in range(lo_bits, hi_bits, CH):
    b = np.arange(start, min(start + CH, hi_bits), dtype=np.uint32)
    x = b.view(np.float32)
    v = vml(x)
    e = ref64(x.astype(np.float64))
    cr = e.astype(np.float32)
    bad = v != cr
    bad &= ~(np.isnan(v) & np.isnan(cr))
    tot += len(x); mism += int(bad.sum())
    # fraction of the exact value between the f32 below it and the f32 above
    a = np.abs(e)
    down = np.abs(cr).astype(np.float64)
    down = np.where(down > a, np.nextafter(np.abs(cr), np.float32(0)).astype(np.float64), down)
    up = np.nextafter(down.astype(np.float32), np.float32(np.inf)).astype(np.float64)
    frac = (a - down) / (up - down)
    fr_mis.append(np.stack([frac[bad], (np.abs(v[bad]).astype(np.float64) - np.abs(cr[bad]))/(up[bad]-down[bad]), x[bad]], 1))
    near = (~bad) & (np.abs(frac - 0.5) < 0.02)
    fr_ok_near.append(frac[near])
print(name, f"{tot} inputs, {mism} differ from correctly rounded ({mism/tot:.4%}) in {time.time()-t0:.0f}s")
m = np.concatenate(fr_mis)
ok = np.concatenate(fr_ok_near)
np.save(f"/tmp/vml/{name}_{sys.argv[2]}_mis.npy", m)
if len(m):
    print(" mismatch frac range", m[:,0].min(), m[:,0].max(), " ulp deltas", np.unique(np.round(m[:,1])))
    print(" frac histogram of mismatches", np.histogram(m[:,0], bins=[0,0.3,0.45,0.49,0.499,0.5,0.501,0.51,0.55,0.7,1])[0])
    print(" matched-near-midpoint frac histogram", np.histogram(ok, bins=[0.48,0.49,0.499,0.4999,0.5,0.5001,0.501,0.51,0.52])[0])
