import sys, os, ctypes as C, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "hip"))
import torch, build_probe
L = C.CDLL(build_probe.build())
fp = C.POINTER(C.c_float)
L.math_probe.argtypes = [C.c_int, C.c_int, fp, fp, fp, fp, C.POINTER(C.c_uint32)]
def run(op, a):
    a = np.ascontiguousarray(a, np.float32); n = a.size
    o0 = np.zeros(n, np.float32); o1 = np.zeros(n, np.float32); u = np.zeros(2*n, np.uint32)
    L.math_probe(op, n, a.ctypes.data_as(fp), a.ctypes.data_as(fp), o0.ctypes.data_as(fp), o1.ctypes.data_as(fp), u.ctypes.data_as(C.POINTER(C.c_uint32)))
    return o0
r = np.random.default_rng(0)
a = np.concatenate([r.uniform(0, 10, 100000), np.abs(r.standard_normal(50000))*1e-3, np.exp(r.uniform(-80, 80, 50000)), r.uniform(0.99, 1.01, 100000), r.random(100000)]).astype(np.float32)
ref = np.sqrt(a)
for op in (2, 9, 10):
    o = run(op, a)
    bad = np.nonzero(o.view(np.uint32) != ref.view(np.uint32))[0]
    print("op", op, "mismatches", len(bad), "of", a.size)
    for i in bad[:8]:
        print("   x=%r gpu=%r ref=%r" % (float(a[i]), float(o[i]), float(ref[i])))
    if len(bad):
        print("   x range of mismatches: min %g max %g" % (a[bad].min(), a[bad].max()))
