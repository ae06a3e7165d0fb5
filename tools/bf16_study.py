import numpy as np, sys
sys.path.insert(0,'/root/repo')
from oracle import emulator as OE
from oracle.dense import dense_predict
import oracle.dense as OD
from fv3net_amd.dense import DenseColumnModel
from fv3net_amd.workloads import dense_2x256_config
b=OE.to_bf16
rng=np.random.default_rng(0)
N=4096
T=(260+15*rng.standard_normal((N,79))).astype(np.float32); q=rng.uniform(0,0.02,(N,79)).astype(np.float32)
m=DenseColumnModel.random(dense_2x256_config(),seed=1,sample_inputs=[T[:64],q[:64]])
P=m.oracle_params()
ref=dense_predict([T,q],P,np.float64)
f32=dense_predict([T,q],P,np.float32)
def split(a):
    a=np.asarray(a,np.float32); h=b(a); l=b(a-h); return h.astype(np.float64),l.astype(np.float64)
def mm3(x,W):
    xh,xl=split(x); wh,wl=split(W); return (xh@wh+xh@wl+xl@wh).astype(np.float32)
# bf16x3 forward
h=np.concatenate([OD.standard_norm(x[:,a:c],mu,s,P["epsilon"],np.float32) for x,(a,c),mu,s in zip([T,q],P["in_clip"],P["in_mean"],P["in_sigma"])],1)
for W,bb in zip(P["hidden_kernels"],P["hidden_biases"]):
    h=np.maximum(mm3(h,W)+bb,0)
outs=[]
for o,(W,bb) in enumerate(zip(P["out_kernels"],P["out_biases"])):
    y=mm3(h,W)+bb; y=y*P["out_sigma"][o]+P["out_mean"][o]; outs.append(y)
for r,g,g2 in zip(ref,outs,f32):
    print("bf16x3",np.abs(g-r).max()/np.abs(r).max(), "f32",np.abs(g2-r).max()/np.abs(r).max())
