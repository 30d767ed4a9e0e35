import sys, numpy as np, multiprocessing as mp, json
sys.path[:0]=['/root/repo/lqr-obstacles_amd','/root/repo/oracle','/root/repo/tests/golden','/root/repo/tests']
N,H,NP,X=16384,200,100,12
R0,R1=int(sys.argv[1]),int(sys.argv[2])
def init():
    global lqro, oracle, models, g0, x, S
    import lqro as _l, pyoracle as _o
    lqro, oracle = _l, _o
    models=lqro.perturbed_models(N); g0=lqro.synthesize_gains(x_dim=X)
    x,_=lqro.synthetic_swarm(N,x_dim=X); S=oracle.sphere(NP)
def row(i):
    gi=lqro.synthesize_gains(models[i],x_dim=X)
    T,NCF=oracle.tables(g0["A"],g0["B"],gi["L"],gi["E"],H,X=X)
    p=x[i,:3]-x[:,:3]; v=x[i,3:6]-x[:,3:6]
    vv=(v*v).sum(1); t=np.where(vv>0,-(p*v).sum(1)/np.where(vv>0,vv,1),0); t=np.clip(t,0,3.0)
    e=p+t[:,None]*v; cand=np.nonzero(((e*e).sum(1)<=9.0)&(np.arange(N)!=i))[0]
    out=[]
    oracle.set_hull_rule(1,round16=True)
    for j in cand:
        rec,idx,pts=oracle.pair(T,NCF,S,x[i],x[j],i,int(j),want_points=True)
        if not (rec["flags"]&2) or rec["n_reach"]<=4: continue
        nf,dist,nrm,fac,qst=oracle.hull_branch_ref(pts,x[i,3:6]-x[j,3:6])
        out.append((i,int(j),int(qst),nf))
    return out
if __name__=="__main__":
    with mp.Pool(8,initializer=init) as pool:
        res=[r for rr in pool.imap_unordered(row,range(R0,R1),chunksize=4) for r in rr]
    json.dump(res,open(f"/tmp/mq/scan_{R0}_{R1}.json","w"))
    q=np.array([r[2] for r in res])
    print("inside",len(res),"merged-fired",int(((q&0xffff)!=0).sum()),"loose",int(((q&0x20000)!=0).sum()),"new",int(((q&0x10000)!=0).sum()))
