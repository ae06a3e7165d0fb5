"""The bench's host-boundary legs alone (bench.host_to_host, rank_call_host_to_host, predict_mappm_host_to_host)."""
import json, sys, os
sys.path.insert(0, os.getcwd())
import torch
import bench
dev = torch.device("cuda", 0)
out = {}
for res in (48, 384):
    out[f"dense_c{res}_host_to_host"] = bench.host_to_host(dev, res)
out["rank_call"] = bench.rank_call_host_to_host(dev)
for rnd in range(2):
    for fence in (True, False):
        out[f"predict_mappm_c384_host_to_host_fence{int(fence)}_{rnd}"] = bench.predict_mappm_host_to_host(dev, fence=fence)
print(json.dumps({k: {kk: v[kk] for kk in v if "ms" in kk} for k, v in out.items()}))
