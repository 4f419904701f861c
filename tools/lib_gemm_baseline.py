import torch, time
dev='cuda'
shapes=[(37759,768,256),(14764,2048,512),(14764,512,2048),(70349,384,128),(90434,288,96),(37759,256,256)]
def t(fn, reps=50):
    fn(); torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)/reps*1e3
for (M,N,K) in shapes:
    r={}
    for dt in (torch.float16, torch.bfloat16, torch.float32):
        a=torch.randn(M,K,device=dev,dtype=dt); w=torch.randn(N,K,device=dev,dtype=dt)
        out=torch.empty(M,N,device=dev,dtype=dt)
        r[str(dt).split('.')[-1]]=t(lambda: torch.matmul(a,w.t(),out=out))
    a=torch.randn(M,K,device=dev,dtype=torch.float16); w=torch.randn(N,K,device=dev,dtype=torch.float16)
    out=torch.empty(M,N,device=dev,dtype=torch.float32)
    # fp16 in, fp32 out via addmm? use out_dtype
    try:
        r['f16->f32']=t(lambda: torch.mm(a,w.t(),out_dtype=torch.float32))
    except Exception as e: r['f16->f32']=str(e)[:40]
    print((M,N,K), {k:(round(v,1) if isinstance(v,float) else v) for k,v in r.items()}, flush=True)
