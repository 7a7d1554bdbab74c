import torch, json
def timeit(fn, iters=20, warm=3):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b)/iters*1000
for M,N,K in [(4096,4096,4096),(8192,8192,8192),(25216,3072,768),(25216,768,3072),(25216,2304,768),(8192,768,3072),(802816,64,64),(802816,64,576)]:
    A=torch.randn(M,K,device='cuda',dtype=torch.bfloat16); B=torch.randn(K,N,device='cuda',dtype=torch.bfloat16)
    us=timeit(lambda: A@B)
    print(json.dumps({"shape":f"torch/hipBLASLt {M}x{N}x{K}","us":round(us,1),"TFLOPs":round(2*M*N*K/us/1e6,1)}))
