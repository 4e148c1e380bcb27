"""Phase breakdown of the persistent 3D kernel (k_ps_slab) from a GP_SLAB_PROF build:

    tools/variants/build.sh prof:-DGP_SLAB_PROF=1
    GP_SLAB_PROF_OUT=/tmp/slab.bin cop5615-gossip_protocol_amd/lib_prof/gossip 100000 3D push-sum --max-rounds 2048
    python3 tools/slab_prof.py /tmp/slab.bin

Workgroup 0 and the middle workgroup stamp s_memrealtime (100 MHz) at 7 points of each round: 0 round
start (compute wave 0; in-block LDS reads done ahead), 1 the neighbours' granules and the lagged gate's
arrival words arrived, 2 round computed into LDS, 3 after the round's barrier (the publisher wave), 4 the
publisher has issued the round's granules, arrival, frozen values and trace."""
import sys

import numpy as np

R, P = 4096, 8
names = ["wait (granules + gate)", "compute -> LDS", "barrier", "publish (publisher wave)"]
t = np.fromfile(sys.argv[1], np.uint64).reshape(2, R, P).astype(np.int64)
for w in range(2):
    x = t[w]
    n = int((x[:, 0] > 0).sum())
    lo, hi = 16, max(17, n - 8)
    x = x[lo:hi]
    d = np.diff(x[:, :5], axis=1) * 10.0 / 1000.0  # us
    per = np.diff(x[:, 0]) * 10.0 / 1000.0
    print(f"workgroup sample {w}: rounds {lo}..{hi - 1}, round period median {np.median(per):.3f} us, mean {per.mean():.3f} us")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} median {np.median(d[:, k]):.3f} us  mean {d[:, k].mean():.3f}")
    print(f"  {'barrier -> next start':22s} median {np.median(x[1:, 0] - x[:-1, 3]) * 0.01:.3f} us")
