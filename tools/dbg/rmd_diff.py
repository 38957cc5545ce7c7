# debug: where do the direct and gather softbuffers differ (GPU box)
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from helpers import make_subframes
from srsue_amd import abi
from test_gpu_parity import CASES

cfgs = [abi.sf_cfg(**c) for c in CASES] + [abi.sf_cfg(**CASES[0]) for _ in range(8)] + \
    [abi.sf_cfg(**CASES[1]) for _ in range(8)]
iqs, _ = make_subframes(cfgs, snr_db=30.0, seed0=41)
res = []
for direct in ("1", "0"):
    os.environ["MI_RM_DIRECT"] = direct
    b = abi.Batch(cfgs, max_its=4, tdec_i16=True, compact_ce=True)
    print("direct groups", b.rm_direct_groups, "groups", b.n_groups)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i, iq in enumerate(iqs):
        flat[2 * b.iq_offset(i):2 * b.iq_offset(i) + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    res.append(b.download(abi.BUF_SB, np.uint32))
    b.close()
a, c = res
bad = np.nonzero(a != c)[0]
print("mismatches", len(bad), "of", len(a))
rows = bad // 64
print("distinct rows", len(np.unique(rows)), "first rows", np.unique(rows)[:20], "last rows", np.unique(rows)[-10:])
for i in bad[:40]:
    print(i, i // 64, i % 64, hex(a[i]), hex(c[i]), a[i:i+1].view(np.float32)[0], c[i:i+1].view(np.float32)[0])
lanes = np.bincount(bad % 64, minlength=64)
print("per lane", lanes.tolist())
