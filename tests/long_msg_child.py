"""TEST HELPER (run by tests/test_long_msg.py in a child process, so the
process-default engine is created with FD_ED25519_GPU_DEFAULT_BLOB set):
the reference-shaped drop-ins over messages longer than that engine's
staging blob.  argv: cases.npz out.json"""
import json
import sys
import threading

import numpy as np

import firedancer_amd as fa

z = np.load(sys.argv[1])
n = int(z["n"])
msgs = [z[f"m{i}"] for i in range(n)]
sigs = [bytes(z["sig"][i]) for i in range(n)]
pubs = [bytes(z["pub"][i]) for i in range(n)]
# fd_ed25519_verify from 4 threads at once (group commit mixes the long
# calls with short ones in shared batches)
per = [None] * n


def worker(t):
    for i in range(t, n, 4):
        per[i] = fa.verify(msgs[i].tobytes(), sigs[i], pubs[i])


th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
for x in th:
    x.start()
for x in th:
    x.join()
r, out = fa.verify_batch([m.tobytes() for m in msgs], sigs, pubs)
sm = z["shared"].tobytes()
rs, outs = fa.verify_batch_single_msg(sm, z["ssig"], z["spub"])
json.dump({"per": per, "batch_r": int(r), "batch": out.tolist(), "single_r": int(rs), "single": outs.tolist(),
           "max_blob": int(fa.lib().fd_ed25519_gpu_max_blob(fa.lib().fd_ed25519_gpu_default()))},
          open(sys.argv[2], "w"))
