import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
from fv3net_amd.mappm import mappm_device
cfg = DenseModelConfig(["T","q"], ["dQ1","dQ2"], [79,79], [79,79], 256, 3)
m = DenseColumnModel.random(cfg, seed=1)
for n in (48, 96, 384):
    T = torch.randn(6, 79, n, n, device='cuda'); q = torch.rand(6, 79, n, n, device='cuda')
    outs = [torch.empty_like(T), torch.empty_like(T)]
    for _ in range(3): m.forward([T, q], [1, 1], outputs=outs, out_level_axis=1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    it = 20
    e0.record()
    for _ in range(it): m.forward([T, q], [1, 1], outputs=outs, out_level_axis=1)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    ncol = 6*n*n
    print(f"dense C{n}: {ms*1e3:.1f} us/step  {ncol/ms*1e3:.3e} col/s  {ncol*cfg.flops_per_column()/ms/1e9:.1f} TFLOP/s")
for (ncol, km, kn) in ((864, 79, 50), (6*384*384, 79, 79)):
    delp = torch.rand(km, ncol, device='cuda') * 1000 + 500
    pe1 = torch.cat([torch.full((1, ncol), 300., device='cuda'), 300 + torch.cumsum(delp, 0)])
    pe2 = pe1.clone() if kn == km else torch.stack([torch.linspace(0,1,kn+1,device='cuda')]*ncol,1) * (pe1[-1]-pe1[0]) + pe1[0]
    q = torch.randn(km, ncol, device='cuda') * 10 + 250
    out = torch.empty(kn, ncol, device='cuda')
    for kord in (1, 10):
        for _ in range(3): mappm_device(pe1, q, pe2, 1, kord, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(20): mappm_device(pe1, q, pe2, 1, kord, out=out)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)/20
        by = (km+1+km+kn+1+kn)*4*ncol
        print(f"mappm ncol={ncol} {km}->{kn} kord={kord}: {ms*1e3:.1f} us  {ncol/ms*1e3:.3e} col/s  {by/ms/1e6:.1f} GB/s")
