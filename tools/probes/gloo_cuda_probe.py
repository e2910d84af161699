import os, torch, torch.distributed as dist
dist.init_process_group("gloo")
r = dist.get_rank()
dev = torch.device("cuda", 0)
x = torch.full((16,), r, dtype=torch.uint8, device=dev)
out = torch.empty(32, dtype=torch.uint8, device=dev)
for name, fn in [("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(out, x)),
                 ("all_to_all_single", lambda: dist.all_to_all_single(torch.empty(16, dtype=torch.uint8, device=dev), x)),
                 ("all_reduce", lambda: dist.all_reduce(torch.ones(4, device=dev)))]:
    try:
        fn(); print(r, name, "ok", flush=True)
    except Exception as e:
        print(r, name, "FAIL", type(e).__name__, str(e)[:100], flush=True)
dist.destroy_process_group()
