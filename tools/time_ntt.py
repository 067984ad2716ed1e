"""Per-kernel timing of the NTT passes (dev tool): python tools/time_ntt.py [log_n] [polys]
Uses FHECORE_LIB to pick an A/B build; prints the average HIP-event time per kernel."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-fhe_amd"))
import torch
import fhecore as fc
from fhecore._capi import load, check
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
polys = int(sys.argv[2]) if len(sys.argv) > 2 else 64
L = 8
ctx = fc.Context(log_n, L=L)
n = 1 << log_n
x = torch.randint(0, 2**59, (polys, L, n), dtype=torch.int64, device="cuda")
a = torch.randint(0, 2**59, (16, 2, L, n), dtype=torch.int64, device="cuda")
b = torch.randint(0, 2**59, (16, 2, L, n), dtype=torch.int64, device="cuda")
for _ in range(3):
    ctx.ntt_(x); ctx.intt_(x); ctx.hommult(a, b)
torch.cuda.synchronize()
lib = load()
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
best = {}
for rep in range(5):  # min over repetitions of the per-kernel mean: damps clock/DVFS noise
    check(lib.fhe_prof_begin(400, st), "prof")
    for _ in range(10):
        ctx.ntt_(x); ctx.intt_(x); ctx.hommult(a, b)
    ms = (ctypes.c_float * 400)(); cnt = ctypes.c_uint32(); names = ctypes.create_string_buffer(16384)
    check(lib.fhe_prof_end(ms, 400, ctypes.byref(cnt), names, 16384), "prof_end")
    per = {}
    for nm, v in zip(names.value.decode().split("\n"), ms[:cnt.value]):
        per.setdefault(nm, []).append(v)
    for k, v in per.items():
        best[k] = min(best.get(k, 1e9), sum(v) / len(v))
tag = os.path.basename(os.environ.get("FHECORE_LIB", "default"))
print(tag, " ".join(f"{k}={v*1000:.1f}us" for k, v in best.items()),
      f"hommult_sum={sum(v for k, v in best.items() if k.startswith('hm_'))*1000:.1f}us")
