"""GPU probe: host time of hipGraphLaunch (torch CUDAGraph.replay) for a graph of K small kernels, alone and with
one RCCL all-reduce (world 1) or a device-to-device copy node captured in it (developer tool, round 4)."""
import os
import time

import torch
import torch.distributed as dist


def graph_of(k, extra):
    side = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")
    y = torch.zeros(1 << 20, device="cuda")
    z = torch.zeros(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
            if extra == "rccl":
                dist.all_reduce(y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for i in range(k):
            x.add_(1.0)
            if extra == "rccl" and i == k // 2:
                dist.all_reduce(y)
            if extra == "copy" and i == k // 2:
                z.copy_(y)
            if extra.startswith("fork") and i % (k // int(extra[4:])) == k // int(extra[4:]) - 1:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    z.add_(1.0)
                    if "rccl" in os.environ.get("PROBE_FORK", ""):
                        dist.all_reduce(z)
                torch.cuda.current_stream().wait_stream(side)
    return g


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    for k in (1000, 3000):
        for extra in ("none", "rccl", "fork1", "fork3", "fork10"):
            g = graph_of(k, extra)
            for idle in (True, False):
                ts = []
                for _ in range(5):
                    if idle:
                        torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    g.replay()
                    ts.append(time.perf_counter() - t0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                gpu = time.perf_counter() - t0
                print(f"K {k:5d} {extra:5s} {'idle GPU' if idle else 'back-to-back'}: replay() host "
                      f"{1e3 * sorted(ts)[2]:.3f} ms (median), replay+sync {1e3 * gpu:.3f} ms", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
