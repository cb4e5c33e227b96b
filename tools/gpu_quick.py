import sys, time, ctypes, numpy as np
sys.path.insert(0, '.')
import firedancer_amd as fa
from firedancer_amd import corpus
t=time.time()
b = corpus.adversarial(6000, 128, seed=3)
print("corpus", time.time()-t, flush=True)
O = ctypes.CDLL('oracle/liboracle.so')
sig,pub,data,off,sz = b.flat()
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
exp = np.zeros(len(b), np.int32)
O.oracle_verify_batch(ctypes.c_uint64(len(b)), P(sig), P(pub), P(data), P(off), P(sz), P(exp), 16)
print("oracle codes", np.unique(exp, return_counts=True), flush=True)
if len(sys.argv) > 1 and sys.argv[1] == 'cpu': sys.exit(0)
e = fa.Engine(0, 1<<16, 1<<24)
t=time.time(); got = e.verify_packed(b.blob, b.desc); print("gpu", time.time()-t, flush=True)
t=time.time(); got = e.verify_packed(b.blob, b.desc); print("gpu2", time.time()-t, flush=True)
mm = np.nonzero(got != exp)[0]
print("mismatches", len(mm), [(int(i), corpus.CASES[b.label[i]], int(exp[i]), int(got[i])) for i in mm[:20]], flush=True)
