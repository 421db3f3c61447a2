import torch, json
def timeit(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ts=[]
    for _ in range(reps):
        a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    ts.sort(); return ts[len(ts)//2]
M=61440
dev='cuda'
for N,K,s in [(3072,1024,4),(1024,1024,8),(8192,1024,2),(1024,4096,4)]:
    g=torch.randn(M,N,device=dev).bfloat16(); x=torch.randn(M,K,device=dev).bfloat16()
    fl=2*M*N*K
    r={"shape":f"N{N}_K{K}_s{s}"}
    r["gT_x_TF"]=round(fl/timeit(lambda: torch.bmm(g.view(s,M//s,N).transpose(1,2), x.view(s,M//s,K), out_dtype=torch.float32))/1e9)
    r["xT_g_TF"]=round(fl/timeit(lambda: torch.bmm(x.view(s,M//s,K).transpose(1,2), g.view(s,M//s,N), out_dtype=torch.float32))/1e9)
    r["gT_x_bf16out_TF"]=round(fl/timeit(lambda: torch.bmm(g.view(s,M//s,N).transpose(1,2), x.view(s,M//s,K)))/1e9)
    r["xT_g_bf16out_TF"]=round(fl/timeit(lambda: torch.bmm(x.view(s,M//s,K).transpose(1,2), g.view(s,M//s,N)))/1e9)
    print(json.dumps(r), flush=True)
