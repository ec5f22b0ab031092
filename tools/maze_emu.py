# CPU emulation of apg_maze.hpp (ring / spill / log / paint) against the reference carve() algorithm.
# emulate apg_maze.hpp's per-lane DFS (ring/spill/log/pad) and paint; compare with the reference algorithm
import numpy as np, sys
T=[0x4e4b272d1b1e3639,0x9c93878d6c637872,0xe4e1d8d2c6c9b4b1]
def perm_of(i): return (T[i//8]>>((i%8)*8))&255
class R:
    def __init__(s,seed): s.g=np.random.default_rng(seed).bit_generator; s.has=0; s.u=0
    def n64(s): return int(s.g.random_raw())
    def n32(s):
        if s.has: s.has=0; return s.u
        v=s.n64(); s.has=1; s.u=v>>32; return v&0xffffffff
    def dbl(s): return (s.n64()>>11)*(1.0/9007199254740992.0)
def draw_perm(r):
    j3=r.n32()&3
    while True:
        j2=r.n32()&3
        if j2<=2: break
    j1=r.n32()&1
    return j3*6+j2*2+j1
RING,CHUNK,PERIOD=64,32,16
def dfs(seed,h,w,bp):
    r=R(seed); ncx=(w-1)//2; ncy=(h-1)//2
    vis=np.zeros((ncy,ncx),bool); vis[0,0]=True
    ring=[0]*RING; spill={}; log=[]; lgbuf=[]
    cx=cy=sp=lo=k=0; frm=0; first=True; done=False; pend=None
    pidx=draw_perm(r); perm=perm_of(pidx)
    stalls=0
    while True:
        for it in range(PERIOD):
            if done: continue
            E=0
            if cx+1<ncx and not vis[cy,cx+1]: E|=1
            if cx-1>=0 and not vis[cy,cx-1]: E|=2
            if cy+1<ncy and not vis[cy+1,cx]: E|=4
            if cy>0 and not vis[cy-1,cx]: E|=8
            pm=0
            for j in range(4): pm|=((E>>((perm>>(2*j))&3))&1)<<j
            pm&=(0xF<<k)&0xF
            if pm:
                j=(pm&-pm).bit_length()-1; d=(perm>>(2*j))&3; k=j+1
                take=first or r.dbl()<bp
                if take:
                    nx=cx+(d==0)-(d==1); ny=cy+(d==2)-(d==3)
                    vis[ny,nx]=True; lgbuf.append(nx|ny<<7|d<<14)
                    assert sp-lo<RING
                    ring[sp%RING]=pidx|frm<<5; sp+=1
                    cx,cy,frm,first,k=nx,ny,d,True,0
                    pidx=draw_perm(r); perm=perm_of(pidx)
            elif sp==0: done=True
            elif sp>lo:
                sp-=1; fb=ring[sp%RING]
                cx-=(frm==0)-(frm==1); cy-=(frm==2)-(frm==3)
                pidx=fb&31; perm=perm_of(pidx)
                k=[((perm>>(2*j))&3)==frm for j in range(4)].index(True)+1
                first=False; frm=fb>>5
            else: stalls+=1
        cnt=sp-lo
        if pend is not None and cnt<=RING-PERIOD-CHUNK:
            for t in range(CHUNK): ring[(lo-CHUNK+t)%RING]=pend[t]
            lo-=CHUNK; pend=None
        elif cnt>RING-PERIOD:
            pend=[ring[(lo+t)%RING] for t in range(CHUNK)]; spill[lo]=list(pend); lo+=CHUNK
        if lgbuf:
            if len(lgbuf)&1: lgbuf.append(0xFFFF)
            log+=lgbuf; lgbuf=[]
        if pend is None and lo>0: pend=list(spill[lo-CHUNK])
        if done: break
    # paint
    m=np.ones((h,w),bool); m[1,1]=False
    for e in log:
        if e==0xFFFF: continue
        x=2*(e&127)+1; y=2*((e>>7)&127)+1; d=e>>14
        m[y,x]=False; m[y-((d==2)-(d==3)), x-((d==0)-(d==1))]=False
    return m,stalls,len(log)
sys.path.insert(0,'/root/repo/oracle')
def ref(idx,h,w,bp):
    rng=np.random.default_rng(idx); maze=np.ones((h,w),bool); dims=np.array([w,h])
    dirs=np.array([[2,0],[-2,0],[0,2],[0,-2]])
    sys.setrecursionlimit(100000)
    def carve(pos):
        first=True
        for dr in rng.permutation(dirs):
            n=pos+dr
            if np.all(0<n) and np.all(n<dims-1) and maze[n[1],n[0]]==1:
                if first or rng.random()<bp:
                    ip=pos+dr//2; maze[ip[1],ip[0]]=False; maze[n[1],n[0]]=False; carve(n); first=False
    maze[1,1]=0; carve(np.ones(2,int)); return maze
import threading
threading.stack_size(512*1024*1024)
def main():
    for (h,w,bp) in [(21,21,1.0),(63,63,1.0),(127,127,1.0),(21,35,0.5),(127,127,0.3),(15,9,0.8)]:
        for idx in [0,1,12345,2**32-1]:
            a,st,nl=dfs(idx,h,w,bp); b=ref(idx,h,w,bp)
            assert np.array_equal(a,b),(h,w,bp,idx)
        print(h,w,bp,'ok stalls',st,'log',nl)
t=threading.Thread(target=main); t.start(); t.join()
