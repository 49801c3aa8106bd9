"""The kv100 Zstd blocks' sequences-section shape, for phase A's LDS window sizes (zstd_fast.hip
zs_fse_parse_kernel): table accuracy logs, header bytes, and the 16-byte chunks each block's section
needs from the chunk holding its first byte and from the one holding its bitstream's first byte.
CPU only: python3 tools/kvwin.py [blocks]."""
import sys, numpy as np, collections
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tools')
import workload as wl
N=int(sys.argv[1]) if len(sys.argv)>1 else 20000
dec, dec_off = wl.decoded_blocks(N, seed=20250307, half=True)
blob, off = wl.encode_blocks(4, dec, dec_off, threads=8)
class BR:
    def __init__(s,b): s.b=b; s.bp=0
    def get(s,n):
        v=0
        for i in range(n):
            byte=s.b[(s.bp+i)>>3] if (s.bp+i)>>3 < len(s.b) else 0
            v|=((byte>>((s.bp+i)&7))&1)<<i
        return v
def ncount(b):
    al=(b[0]&15)+5; bp=4; rem=(1<<al)+1; thr=1<<al; nb=al+1; s=0; prev0=False
    r=BR(b)
    while rem>1:
        if prev0:
            n0=s
            while True:
                r.bp=bp; v=r.get(2); bp+=2; n0+=v
                if v!=3: break
            s=n0; prev0=False
        r.bp=bp; v=r.get(nb); mx=(2*thr-1)-rem
        if (v&(thr-1))<mx: c=v&(thr-1); bp+=nb-1
        else:
            c=v&(2*thr-1)
            if c>=thr: c-=mx
            bp+=nb
        c-=1; rem-= -c if c<0 else c; s+=1; prev0=c==0
        while rem<thr and nb>1: nb-=1; thr>>=1
    return (bp+7)//8, al
stats=collections.Counter(); need12=[]; need_after=[]; als=collections.Counter(); hdr=[]; nseqs=[]
for i in range(N):
    f=bytes(blob[int(off[i]):int(off[i+1])]); shift=int(off[i])&15
    assert f[:4]==b'\x28\xb5\x2f\xfd'
    fhd=f[4]; fcsf=fhd>>6; ss=(fhd>>5)&1; ck=(fhd>>2)&1; did=fhd&3
    p=5+(0 if ss else 1)+[0,1,2,4][did]+([1 if ss else 0,2,4,8][fcsf])
    bh=f[p]|f[p+1]<<8|f[p+2]<<16; bt=(bh>>1)&3; bs=bh>>3; body=p+3
    if bt!=2: stats['bt%d'%bt]+=1; continue
    b0=f[body]; lt=b0&3; sf=(b0>>2)&3
    if lt>1: stats['huflit']+=1; continue
    if sf==1: hs=2; nlit=(b0>>4)+(f[body+1]<<4)
    elif sf==3: hs=3; nlit=(b0>>4)+(f[body+1]<<4)+(f[body+2]<<12)
    else: hs=1; nlit=b0>>3
    pos=hs+(nlit if lt==0 else 1); s=body+pos
    c0=f[s]
    if c0<128: nseq=c0; sp=1
    elif c0<255: nseq=((c0-128)<<8)+f[s+1]; sp=2
    else: nseq=f[s+1]+(f[s+2]<<8)+0x7f00; sp=3
    modes=f[s+sp]; sp+=1
    ms=[modes>>6,(modes>>4)&3,(modes>>2)&3]; al=[]
    for m,d in zip(ms,[6,5,6]):
        if m==2:
            u,a=ncount(f[s+sp:]); sp+=u; al.append(a)
        elif m==1: sp+=1; al.append(0)
        elif m==0: al.append(d)
        else: al.append(-1)
    als[tuple(al)]+=1; hdr.append(sp); nseqs.append(nseq)
    end=body+bs+(4 if ck else 0)
    c_lo=(shift+s)>>4
    need12.append(((shift+end+15)>>4)-c_lo)   # chunks needed from c_lo (wend = 16*(c_lo+K)-shift >= end)
    c_lo2=(shift+s+sp)>>4
    need_after.append(((shift+end+15)>>4)-c_lo2)
def dist(x):
    x=np.array(x); return {k:int((x>k).sum()) for k in (8,9,10,11,12)}
print('N',N,stats,'nseq mean',np.mean(nseqs),'max',max(nseqs),'hdr mean',np.mean(hdr),'max',max(hdr))
print('tables',als.most_common(8))
print('chunks needed from c_lo: >K counts',dist(need12), 'max',max(need12))
print('chunks needed from bitstream start: >K counts',dist(need_after),'max',max(need_after))
