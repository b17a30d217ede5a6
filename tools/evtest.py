import sys, time, torch, numpy as np
sys.path.insert(0, '/root/repo')
from ugo_amd import fec
d,p,S,G=10,3,1350,65536; n=13; pitch=1360
enc=fec.New(d,p)
gen=torch.Generator(device='cuda').manual_seed(1)
sh=torch.randint(0,256,(n,G,pitch),dtype=torch.uint8,device='cuda',generator=gen)
rng=np.random.default_rng(2)
m=np.full(G,(1<<n)-1,np.uint64)
for g in range(G):
    a,b=rng.choice(n,2,replace=False); m[g]&=~np.uint64((1<<int(a))|(1<<int(b)))
masks=torch.as_tensor(m.view(np.int64)).cuda()
s=torch.cuda.current_stream()
def step(ev=None):
    if ev: ev[0].record(s)
    enc.encode_batch(sh,S,shard_major=True)
    if ev: ev[1].record(s)
    enc.reconstruct_batch(sh,masks,S,shard_major=True)
    if ev: ev[2].record(s)
for _ in range(5): step()
torch.cuda.synchronize()
for mode in ("noev","ev","noev","ev"):
    K=50
    evs=[[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)] if mode=="ev" else [None]*K
    torch.cuda.synchronize(); t=time.perf_counter()
    for k in range(K): step(evs[k])
    torch.cuda.synchronize(); el=(time.perf_counter()-t)/K*1e6
    extra=""
    if mode=="ev":
        e=sum(x[0].elapsed_time(x[1]) for x in evs)/K*1e3; r=sum(x[1].elapsed_time(x[2]) for x in evs)/K*1e3
        extra=f" enc {e:.1f} rec {r:.1f}"
    print(mode, f"{el:.1f} us/step"+extra, flush=True)
# only reconstruct back to back
for mode in ("rec-only-noev","rec-only-ev"):
    K=50
    torch.cuda.synchronize(); t=time.perf_counter()
    evs=[[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(K)]
    for k in range(K):
        if mode.endswith("-ev"): evs[k][0].record(s)
        enc.reconstruct_batch(sh,masks,S,shard_major=True)
        if mode.endswith("-ev"): evs[k][1].record(s)
    torch.cuda.synchronize(); el=(time.perf_counter()-t)/K*1e6
    extra=""
    if mode.endswith("-ev"): extra=f" ev-avg {sum(x[0].elapsed_time(x[1]) for x in evs)/K*1e3:.1f}"
    print(mode, f"{el:.1f} us/launch"+extra, flush=True)
