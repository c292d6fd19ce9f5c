import sys; import os; sys.path[:0] = [os.getcwd(), os.getcwd() + "/tests"]
import ctypes, numpy as np
import soundchunks_amd as sc
lib = sc.load()
FP = ctypes.POINTER(ctypes.c_float)
a = np.random.default_rng(1).normal(size=(32, 16)).astype(np.float32)
pa = (FP * 32)(*[ctypes.cast(a.ctypes.data + i * 64, FP) for i in range(32)])
t = lib.ann_kdtree_create(pa, 32, 16, 1, 0)
print("tree", t, flush=True)
e = ctypes.c_float()
print("search", lib.ann_kdtree_search(t, ctypes.cast(a.ctypes.data, FP), 0.0, ctypes.byref(e)), e.value)
lib.ann_kdtree_destroy(t)
