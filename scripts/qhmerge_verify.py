import sys, json, numpy as np, multiprocessing as mp
sys.path[:0]=['/root/repo/lqr-obstacles_amd','/root/repo/oracle','/root/repo/tests/golden','/root/repo/tests']
N,H,NP,X=16384,200,100,12
def init():
    global lqro, oracle, models, g0, x, S, qhull_lib, reference_rule
    import lqro as _l, pyoracle as _o, qhull_lib as _q
    from make_golden_merge import reference_rule as rr
    lqro, oracle, qhull_lib, reference_rule = _l, _o, _q, rr
    models=lqro.perturbed_models(N); g0=lqro.synthesize_gains(x_dim=X)
    x,_=lqro.synthetic_swarm(N,x_dim=X); S=oracle.sphere(NP)
def one(p):
    i,j,qst,nf=p
    gi=lqro.synthesize_gains(models[i],x_dim=X)
    T,NCF=oracle.tables(g0["A"],g0["B"],gi["L"],gi["E"],H,X=X)
    rec,idx,pts=oracle.pair(T,NCF,S,x[i],x[j],i,j,want_points=True)
    vrel=x[i,3:6]-x[j,3:6]
    rounded=np.array([[oracle.round6(v) for v in row] for row in pts])
    planes,fv,_,_=qhull_lib.qconvex(rounded)
    best,d,stale,nrm=reference_rule(pts,planes,fv,vrel)
    oracle.set_hull_rule(1,round16=True)
    onf,dist,onrm,fac,q2=oracle.hull_branch_ref(pts,vrel)
    same = (d==dist) and (stale==(onrm is None)) and (stale or np.array_equal(nrm,onrm))
    return (i,j,qst,len(fv[best])>3,sum(len(f)>3 for f in fv),bool(same))
if __name__=="__main__":
    r=json.load(open('/tmp/mq/scan_0_16384.json'))
    new=[p for p in r if p[2]&0x10000]
    loose=[p for p in r if (p[2]&0x20000) and not (p[2]&0x10000)]
    rng=np.random.default_rng(0)
    pick=new+[loose[k] for k in rng.choice(len(loose),min(len(loose),int(sys.argv[1])),replace=False)]
    with mp.Pool(8,initializer=init) as pool:
        out=pool.map(one,pick)
    for o in out: print(o)
    print("winner merged:",sum(o[3] for o in out),"results differ:",sum(not o[5] for o in out),"of",len(out))
