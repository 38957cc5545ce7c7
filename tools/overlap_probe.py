"""Probe: do consecutive batches overlap on two streams?  Two workspaces (abi.Batch) of the headline shard,
steps alternated over two HIP streams, against the single-stream loop.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from srsue_amd import abi  # noqa: E402


def main():
    B, P, steps = 12500, 256, 10
    dev = torch.device("cuda", 0)
    cfgs = bench.config_cfgs(4, B, 0)
    pool_iq, pool_tb = bench.make_pool(cfgs[:P], 30.0, 16, 0, None)
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    batches = [abi.Batch(cfgs, max_its=4) for _ in range(nb)]
    d_iq = torch.empty(2 * batches[0].iq_samples, dtype=torch.float32, device=dev)
    sfl = len(pool_iq[0])
    d_pool = torch.from_numpy(np.stack(pool_iq)).to(dev)
    d_iq.view(B, sfl).copy_(d_pool[torch.arange(B, device=dev) % P])
    streams = [torch.cuda.Stream(dev) for _ in range(nb)]
    out = {}
    for mode in ("one", "multi"):
        for w in range(2):
            for i in range(nb):
                batches[i].run(d_iq.data_ptr(), streams[i].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(steps * (nb if mode == "multi" else 1)):
            i = s % nb if mode == "multi" else 0
            batches[i].run(d_iq.data_ptr(), streams[i].cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        n = steps * (nb if mode == "multi" else 1)
        out[mode] = {"steps": n, "ms_per_step": round(el / n * 1e3, 3), "Gbps": round(n * B * 75376 / el / 1e9, 2)}
    for i in range(nb):
        crc = batches[i].download(abi.BUF_TB_CRC, np.uint32)[:B]
        out[f"crc_ok_{i}"] = float(crc.mean())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
