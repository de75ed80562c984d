# CPU model of k_infl_scan1 / k_infl_scan2 (zgpu_inflate.hip): a pure-Python block walker lists the true
# block headers of zlib streams; every true stored / dynamic header must pass both filters, and the
# survivors are counted.  Run from the repository root.
import sys, zlib, numpy as np
sys.path.insert(0, 'tests'); import datagen
ORDER=[16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
class BR:
    def __init__(s, b, pos): s.b=b; s.pos=pos
    def get(s, k):
        v=0
        for i in range(k):
            p=s.pos+i; v |= ((s.b[p>>3]>>(p&7))&1)<<i
        s.pos+=k; return v
def build(lens):
    cnt=[0]*16
    for l in lens: cnt[l]+=1
    cnt[0]=0
    syms=sorted([(l,i) for i,l in enumerate(lens) if l])
    return cnt,[i for l,i in syms]
def dec(r, h):
    cnt,sym=h; code=first=index=0
    for l in range(1,16):
        code|=r.get(1); c=cnt[l]
        if code-first < c: return sym[index+code-first]
        index+=c; first+=c; first<<=1; code<<=1
    raise ValueError
LB=[3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE=[0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DE=[0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
def blocks(z, start):
    r=BR(z,start); out=[]
    while True:
        b=r.pos; last=r.get(1); t=r.get(2); out.append((b,t))
        if t==0:
            r.pos=(r.pos+7)&~7; ln=r.get(16); r.get(16); r.pos+=8*ln
        else:
            if t==1:
                L=build([8]*144+[9]*112+[7]*24+[8]*8); D=build([5]*30)
            else:
                nl=r.get(5)+257; nd=r.get(5)+1; nc=r.get(4)+4
                cl=[0]*19
                for i in range(nc): cl[ORDER[i]]=r.get(3)
                C=build(cl); lens=[]
                while len(lens)<nl+nd:
                    s=dec(r,C)
                    if s<16: lens.append(s)
                    elif s==16: lens+= [lens[-1]]*(3+r.get(2))
                    elif s==17: lens+=[0]*(3+r.get(3))
                    else: lens+=[0]*(11+r.get(7))
                L=build(lens[:nl]); D=build(lens[nl:])
            while True:
                s=dec(r,L)
                if s<256: continue
                if s==256: break
                r.get(LE[s-257]); d=dec(r,D); r.get(DE[d])
        if last: return out
def scan1(z, b0):
    n=len(z); nb=8*n
    bits=np.unpackbits(np.frombuffer(z,np.uint8), bitorder='little').astype(np.uint64)
    pad=np.concatenate([bits, np.zeros(128,np.uint64)])
    def field(off, k):
        v=np.zeros(nb-b0,np.uint64)
        for i in range(k): v |= pad[b0+off+i: b0+off+i+nb-b0] << np.uint64(i)
        return v
    t=field(1,2); hlit=field(3,5); hdist=field(8,5); hcl=field(13,4)+4
    kr=np.zeros(nb-b0,np.uint64)
    for i in range(19):
        l=field(17+3*i,3)
        kr += np.where((l>0)&(i<hcl), np.uint64(128)>>np.minimum(l,7), 0)
    dyn=(t==2)&(hlit<=29)&(hdist<=29)&(kr==128)
    cand=set((np.nonzero(dyn)[0]+b0).tolist())
    # stored
    st=np.nonzero(t==0)[0]+b0
    for b in st.tolist():
        p=(b+3+7)>>3
        if p+4<=n:
            ln=z[p]|z[p+1]<<8; nl=z[p+2]|z[p+3]<<8
            if ln==nl^0xffff and p+4+ln<=n: cand.add(b)
    return cand
def scan2(z, b):
    r=BR(z+bytes(64), b); h=r.get(3)
    if (h>>1)&3!=2: return True
    nl=r.get(5)+257; nd=r.get(5)+1; nc=r.get(4)+4
    cl=[0]*19
    for i in range(nc): cl[ORDER[i]]=r.get(3)
    C=build(cl); lens=[]
    try:
        while len(lens)<nl+nd:
            s=dec(r,C)
            if s<16: lens.append(s)
            elif s==16:
                if not lens: return False
                lens+= [lens[-1]]*(3+r.get(2))
            elif s==17: lens+=[0]*(3+r.get(3))
            else: lens+=[0]*(11+r.get(7))
    except ValueError: return False
    if len(lens)>nl+nd: return False
    def ok(ls):
        k=sum(1<<(15-l) for l in ls if l); mx=max(ls+[0])
        return k<=32768 and (k==32768 or mx<=1)
    lit=lens[:nl]; dist=lens[nl:]
    return lit[256]!=0 and ok(lit) and ok(dist) and r.pos <= 8*len(z)
for kind,level,strat in (("mix",6,0),("text",1,0),("mix",6,4),("runs",9,0),("mix",0,0)):
    data=b"".join(datagen.make(k,150000,7) for k in ("text",kind,"runs"))
    c=zlib.compressobj(level,8,15,8,strat); z=c.compress(data)+c.flush()
    true=blocks(z,16)
    c1=scan1(z,16)
    miss=[(b,t) for b,t in true if t!=1 and b not in c1]
    c2=[b for b in sorted(c1) if scan2(z,b)]
    miss2=[(b,t) for b,t in true if t!=1 and b not in c2]
    print(kind,level,strat,"len",len(z),"blocks",len(true),"types",sorted(set(t for b,t in true)),"scan1",len(c1),"miss1",len(miss),"scan2",len(c2),"miss2",len(miss2))
