# CPU simulation of k_traverse4's walk work (quad visits, triangle tests per ray) without and with the
# exact t-cull margins (build_qcull via pt_scene_bvh_tcull), on the tessellated-mesh scene or config 5;
# also asserts the closest hit is the same in every mode.  usage: python scripts/sim_tcull.py tess|cfg5 NRAYS
# Simulate k_traverse4's walk with/without the exact t-cull (child cull; + pop-time cull) on CPU:
# counts quad visits and triangle tests per ray, checks the result equals the reference walk.
import sys, numpy as np, ctypes as C
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import _native as N, scenes
import test_bvh_quads_cpu as QT
import test_tcull_cpu as TC
f32=np.float32
which=sys.argv[1]
path = scenes.tessellated_meshes('/tmp/tc/sim', res=(64,36)) if which=='tess' else scenes.random_triangles('/tmp/tc/sim5', n=100_000, res=(64,36), depth=32)
s,frac,W,_,tv=TC._tcull_tables(path)
pn,Q,root,bound=QT._tables(s)
A=(W & 0xffff).astype(np.uint16).view(np.float16).astype(np.float64)
B=(W >> 16).astype(np.uint16).view(np.float16).astype(np.float64)
IDX=QT.IDX_MASK
def walk(o,d,mode):
    # mode 0 none, 1 child cull, 2 child + pop cull
    inv=(f32(1)/d).astype(f32); negm=int(d[0]<0)|(int(d[1]<0)<<1)|(int(d[2]<0)<<2)
    best=np.inf; bi=-1; nq=nt=0
    if not QT._slab(pn[0]["bmin"], pn[0]["bmax"], o, inv, True): return best,bi,0,0
    stack=[]; code=root
    while True:
        if code<0:
            c=-code-1; t0=c>>8; cnt=c&255
            for t in range(t0,t0+cnt):
                nt+=1
                h=TC._ray_tri(tv[t][0],tv[t][1],tv[t][2],o,d)
                if h is not None and float(h[2])<best: best=float(h[2]); bi=t
        else:
            qi=code&IDX; q=Q[qi]; nq+=1
            meta=(code>>21)&1023
            hm=0; thr=[-np.inf]*4
            for k in range(4):
                lo=np.array([q["lox"][k],q["loy"][k],q["loz"][k]],f32); hi=np.array([q["hix"][k],q["hiy"][k],q["hiz"][k]],f32)
                if (meta>>k)&1 and QT._slab(lo,hi,o,inv,True):
                    sv=np.where(d<0,hi,lo).astype(f32); t=((sv-o).astype(f32)*d).astype(f32)
                    lo_=float(f32(f32(f32(t[0]+t[1])+t[2]) - f32(f32(f32(abs(t[0])+abs(t[1]))+abs(t[2]))*f32(2**-20))))
                    th=A[qi,k]*lo_*(1-2**-20)/(1+2**-20)-B[qi,k] if lo_>0 else -np.inf
                    thr[k]=th
                    if mode>=1 and th>best: continue
                    hm|=1<<k
            c=[(int(x),thr[i]) for i,x in enumerate(q["code"])]
            if (negm>>((meta>>6)&3))&1:
                c[0],c[1]=c[1],c[0]; hm=(hm&12)|((hm&1)<<1)|((hm>>1)&1)
            if (negm>>((meta>>8)&3))&1:
                c[2],c[3]=c[3],c[2]; hm=(hm&3)|((hm&4)<<1)|((hm>>1)&4)
            if (negm>>((meta>>4)&3))&1:
                c=[c[2],c[3],c[0],c[1]]; hm=((hm&3)<<2)|(hm>>2)
            hits=[c[k] for k in range(4) if (hm>>k)&1]
            if hits:
                stack.extend(reversed(hits[1:])); code=hits[0][0]; continue
        while True:
            if not stack: return best,bi,nq,nt
            code,th=stack.pop()
            if mode==2 and th>best: continue
            break
rng=np.random.default_rng(3)
# rays: camera-like toward the mesh region + from random points in the room
N_=int(sys.argv[2]); res={0:[0,0,0],1:[0,0,0],2:[0,0,0]}
lo_r=pn[0]["bmin"].astype(np.float64); hi_r=pn[0]["bmax"].astype(np.float64)
for i in range(N_):
    tgt=rng.uniform(lo_r,hi_r)
    if i%2==0: o=np.array([0,5,10.5])+rng.normal(0,0.3,3)
    else: o=rng.uniform((-4.9,0.1,-4.9),(4.9,9.9,4.9))
    d=tgt-o; d/=np.linalg.norm(d)
    o=o.astype(f32); d=d.astype(f32)
    ref=None
    for m in (0,1,2):
        b,bi,nq,nt=walk(o,d,m)
        if ref is None: ref=(b,bi)
        else: assert (b,bi)==ref, (m,b,bi,ref)
        res[m][0]+=1; res[m][1]+=nq; res[m][2]+=nt
for m in (0,1,2): print(which, ["no cull","child cull","child+pop cull"][m], "quads/ray", round(res[m][1]/N_,1), "tris/ray", round(res[m][2]/N_,1))
