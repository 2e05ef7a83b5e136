import sys, time, os
sys.path[:0]=['/root/repo/sdn-mpi-router_amd','/root/repo']
import numpy as np, torch
from sdnmpi_amd import _native, topologies as T
from oracle import oracle as O
f=T.fat_tree(48); csr=f.csr(); V=csr.V; H=f.n_hosts
hv,hp=f.host_table(); srcs=np.unique(hv).astype(np.int32); S=len(srcs)
dev=torch.device('cuda',0); st=torch.cuda.Stream(dev); torch.cuda.set_stream(st)
ctx=_native.Context(0); ctx.upload(csr); ctx.set_stream(st.cuda_stream)
ts=torch.from_numpy(srcs).to(dev)
par=torch.empty((S,V),dtype=torch.int32,device=dev); prt=torch.empty_like(par); hop=torch.empty_like(par)
ctx.dfs_tables_device(ts.data_ptr(),S,par.data_ptr(),prt.data_ptr(),hop.data_ptr()); ctx.synchronize()
ml=int(hop.max().item())+1; print('max_len',ml)
n=1<<22
rng=np.random.default_rng(1); a=rng.integers(0,H,n); b=rng.integers(0,H,n)
rows=torch.from_numpy(np.searchsorted(srcs,hv[a]).astype(np.int32)).to(dev)
dsts=torch.from_numpy(hv[b].astype(np.int32)).to(dev); last=torch.from_numpy(hp[b].astype(np.int32)).to(dev)
off=torch.empty(n+1,dtype=torch.int64,device=dev)
sw=torch.empty(n*ml,dtype=torch.int32,device=dev); hpo=torch.empty_like(sw)
for rep in range(3):
    torch.cuda.synchronize(); t0=time.perf_counter()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True); e0.record(st)
    ctx.route_offsets_device(hop.data_ptr(),rows.data_ptr(),dsts.data_ptr(),n,off.data_ptr(),nrows=S)
    ctx.expand_routes_device(par.data_ptr(),prt.data_ptr(),S,rows.data_ptr(),dsts.data_ptr(),last.data_ptr(),n,off.data_ptr(),sw.data_ptr(),hpo.data_ptr(),timing=True)
    e1.record(st); torch.cuda.synchronize(); ctx.synchronize()
    print('wall %.3f ms  events %.3f ms  kernel %.3f ms  entries %d' % ((time.perf_counter()-t0)*1e3, e0.elapsed_time(e1), ctx.last_kernel_ms(), int(off[-1].item())))
# verify some pairs
o=off.cpu().numpy(); swh=sw.cpu().numpy(); hph=hpo.cpu().numpy()
po,to,_=O.dfs_tables(csr,srcs,with_hops=False,nthreads=16)
bad=0
for i in rng.integers(0,n,2000):
    r=np.searchsorted(srcs,hv[a[i]]); want=O.tree_fdb(csr,po[r],to[r],int(hv[a[i]]),int(hv[b[i]]),hp[b[i]])
    got=[(int(csr.dpids[x]),int(y)) for x,y in zip(swh[o[i]:o[i+1]],hph[o[i]:o[i+1]])]
    bad+= got!=want
print('bad',bad)
