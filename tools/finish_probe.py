"""Profiling aid: the loop iteration at which each block of a 262 k-block V-half batch
finishes (SLATE_DEBUG_MODE 131072 stores it in meta.detail), against the length of its
64-block round: the lockstep tail (rounds wait for their slowest lane)."""
import json,sys,os
sys.path[:0]=['/root/repo','/root/repo/slatedb-go_amd']
import numpy as np, torch
import slatecodec as sc
from tools import workload as wl
n=262144
blob,in_off,dec=wl.snappy_vhalf(n)
dev=torch.device('cuda',0); s=torch.cuda.Stream(dev); ctx=sc.Context(0); ctx.set_stream(s.cuda_stream)
with torch.cuda.stream(s):
    d_in=torch.from_numpy(blob).to(dev); d_off=torch.from_numpy(in_off.view(np.int64)).to(dev)
    d_oo=torch.empty(n+1,dtype=torch.int64,device=dev); d_rb=torch.empty(n+1,dtype=torch.int64,device=dev)
    d_sc=torch.empty(sc.decode_scratch_bytes(n)+64,dtype=torch.uint8,device=dev)
    ctx.decode_plan_device(1,d_in.data_ptr(),d_off.data_ptr(),n,d_oo.data_ptr(),d_rb.data_ptr(),d_sc.data_ptr()); s.synchronize()
    d_out=torch.empty(int(d_oo[n].item())+16,dtype=torch.uint8,device=dev); d_meta=torch.empty(n*16,dtype=torch.uint8,device=dev)
    d_rows=torch.empty(int(d_rb[n].item())*16+16,dtype=torch.uint8,device=dev)
    os.environ['SLATE_DEBUG_MODE']=str(131072)
    ctx.decode_device(1,d_in.data_ptr(),d_off.data_ptr(),n,d_out.data_ptr(),d_oo.data_ptr(),d_meta.data_ptr(),d_rows.data_ptr(),d_rb.data_ptr()); s.synchronize()
meta=np.frombuffer(d_meta.cpu().numpy().tobytes(),dtype=sc.META_DTYPE)
f=meta['detail'].astype(np.float64).reshape(-1,64)
# what grouping similar blocks into rounds could give: rounds formed after sorting by the block's
# own finish (the bound) or by its encoded length (known before decoding)
fl=f.reshape(-1)
clen=np.diff(in_off.astype(np.int64))
by_fin=np.sort(fl).reshape(-1,64).max(axis=1).mean()
by_len=fl[np.argsort(clen,kind="stable")].reshape(-1,64).max(axis=1).mean()
print(json.dumps({"mean_block_finish":float(f.mean()),"mean_round_max":float(f.max(axis=1).mean()),"median_block":float(np.median(f)),
 "p90_block":float(np.percentile(f,90)),"mean_round_min":float(f.min(axis=1).mean()),
 "round_max_if_sorted_by_finish":float(by_fin),"round_max_if_sorted_by_len":float(by_len),
 "corr_len_finish":float(np.corrcoef(clen,fl)[0,1])}))
