#!/usr/bin/env python3
"""Probe for VERDICT r01 weak 7: does a HIP stream forked from an already
forked stream break hipGraph capture (ROCm 7.2, torch 2.10)?

Each variant captures one torch.cuda.CUDAGraph whose body forks main ->
side1 -> side2, runs kernels on every stream, joins back, ends the capture,
replays it and checks the numbers. Variants isolate what the product's
nested branch (dmf_ops.branch inside train_fusion._encode's DCE stream) does:
allocating from the graph pool on the nested stream, freeing that block
before / after the join, record_stream on it, joining side2 directly into
main. Every variant runs in its own child process (a failed capture can leave
the process unusable), bounded by a timeout; one JSON line per variant.

    python tools/capture_fork_probe.py [variant ...]
"""
import json
import subprocess
import sys

VARIANTS = ["flat_fork", "nested_no_alloc", "nested_alloc_free_after_join", "nested_alloc_free_before_join",
            "nested_alloc_record_stream", "nested_join_to_main", "nested_alloc_kept", "nested_reused_side",
            "nested_persistent_events", "nested_keep_graph", "nested_inplace_only", "flat_inplace_only",
            "nested_raw_capture",
            "rccl_capture", "rccl_capture_side_stream"]


def run_rccl(name):
    """all_reduce captured into a hipGraph on a 1-rank RCCL communicator
    (the only RCCL group one GPU allows), on the capture stream or on a side
    stream forked inside the capture (the overlap design)."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        x = torch.full((1 << 20,), 3.0, device=dev)
        comm = torch.cuda.Stream(dev)

        def body():
            x.mul_(2.0)
            if name == "rccl_capture":
                dist.all_reduce(x)
            else:
                cur = torch.cuda.current_stream()
                comm.wait_stream(cur)
                with torch.cuda.stream(comm):
                    dist.all_reduce(x)
                cur.wait_stream(comm)
            x.add_(1.0)

        main = torch.cuda.Stream(dev)
        with torch.cuda.stream(main):
            body()            # eager warm-up: communicator init outside capture
        torch.cuda.synchronize()
        x.fill_(3.0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main):
            body()
        x.fill_(3.0)
        g.replay()
        torch.cuda.synchronize()
        got = float(x[0].item())
        return {"variant": name, "ok": got == 7.0, "value": got, "want": 7.0}
    finally:
        dist.destroy_process_group()


def run_variant(name):
    if name.startswith("rccl"):
        return run_rccl(name)
    import torch

    dev = torch.device("cuda", 0)
    main = torch.cuda.Stream(dev)
    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)
    x = torch.ones(1 << 20, device=dev)
    out = torch.zeros_like(x)
    kept = []

    evs = [torch.cuda.Event() for _ in range(4)]  # nested_persistent_events: alive past capture end

    def wait(dst, src, i):
        if name == "nested_persistent_events":
            evs[i].record(src)
            dst.wait_event(evs[i])
        else:
            dst.wait_stream(src)  # torch: a temporary event, freed right after the wait

    y = torch.zeros_like(x)

    def body_inplace():
        # no allocation anywhere in the capture: only in-place kernels on
        # tensors made before it, still forked main -> s1 (-> s2)
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        with torch.cuda.stream(s1):
            y.copy_(x).mul_(2.0)
            if name.startswith("nested"):
                s2.wait_stream(s1)
                with torch.cuda.stream(s2):
                    y.mul_(3.0)
                s1.wait_stream(s2)
            y.add_(1.0)
        cur.wait_stream(s1)
        out.copy_(y)

    def body_inplace_nested():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        with torch.cuda.stream(s1):
            y.copy_(x).mul_(2.0)
            s2.wait_stream(s1)
            with torch.cuda.stream(s2):
                y.mul_(3.0)
            s1.wait_stream(s2)
            y.add_(1.0)
        cur.wait_stream(s1)
        out.copy_(y)

    def body():
        if name == "nested_raw_capture":
            return body_inplace_nested()
        if name.endswith("inplace_only"):
            return body_inplace()
        cur = torch.cuda.current_stream()
        wait(s1, cur, 0)
        with torch.cuda.stream(s1):
            a = x * 2.0                      # graph-pool block made on s1
            if name == "flat_fork":
                b = a + 1.0
            else:
                wait(s2, s1, 1)              # the nested fork
                with torch.cuda.stream(s2):
                    if name in ("nested_no_alloc", "nested_persistent_events", "nested_keep_graph"):
                        out.add_(a)          # no allocation on s2
                        b = a
                    else:
                        t = a * 3.0          # allocation on s2
                        if name == "nested_alloc_record_stream":
                            t.record_stream(s1)
                        if name == "nested_alloc_kept":
                            kept.append(t)
                        b = t + 0.0
                if name == "nested_join_to_main":
                    pass
                else:
                    wait(s1, s2, 2)
                if name == "nested_alloc_free_before_join":
                    del t
                if name == "nested_reused_side":
                    # fork the same nested stream a second time
                    s2.wait_stream(s1)
                    with torch.cuda.stream(s2):
                        b = b * 1.0
                    s1.wait_stream(s2)
            c = b + 1.0
        if name == "nested_join_to_main":
            cur.wait_stream(s2)
        wait(cur, s1, 3)
        out.copy_(c)

    torch.cuda.synchronize()
    with torch.cuda.stream(main):
        for _ in range(2):
            body()
    torch.cuda.synchronize()
    if name == "nested_raw_capture":
        # the same torch kernels and stream waits, captured with the HIP API
        # directly (ctypes) instead of torch.cuda.CUDAGraph
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        vp = ctypes.c_void_p
        graph, exe = vp(), vp()
        ms = vp(main.cuda_stream)
        assert hip.hipStreamBeginCapture(ms, 0) == 0
        with torch.cuda.stream(main):
            body_inplace_nested()
        rc = hip.hipStreamEndCapture(ms, ctypes.byref(graph))
        assert rc == 0, f"hipStreamEndCapture -> {rc}"
        assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
        out.zero_()
        torch.cuda.synchronize()
        assert hip.hipGraphLaunch(exe, ms) == 0
        torch.cuda.synchronize()
        got = float(out[0].item())
        return {"variant": name, "ok": got == 7.0, "value": got, "want": 7.0}
    g = torch.cuda.CUDAGraph(keep_graph=name == "nested_keep_graph")
    with torch.cuda.graph(g, stream=main):
        body()
    if name == "nested_keep_graph":
        print("capture ended; instantiating", file=sys.stderr, flush=True)
        g.instantiate()
        print("instantiated", file=sys.stderr, flush=True)
    g.replay()
    torch.cuda.synchronize()
    want = {"flat_fork": 4.0, "nested_no_alloc": 3.0, "nested_persistent_events": 3.0, "nested_keep_graph": 3.0,
            "flat_inplace_only": 3.0}.get(name, 7.0)
    got = float(out[0].item())
    return {"variant": name, "ok": abs(got - want) < 1e-6, "value": got, "want": want}


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        try:
            print(json.dumps(run_variant(sys.argv[2])))
        except Exception as e:  # report, do not re-raise: the parent records the line
            print(json.dumps({"variant": sys.argv[2], "ok": False, "error": f"{type(e).__name__}: {e}"[:400]}))
        return
    names = sys.argv[1:] or VARIANTS
    for n in names:
        try:
            r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, "--child", n], capture_output=True, text=True, timeout=120)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            res = json.loads(line[-1]) if line else {"variant": n, "ok": False, "rc": r.returncode,
                                                     "stderr": r.stderr[-1500:]}
            res["rc"] = r.returncode
        except subprocess.TimeoutExpired:
            res = {"variant": n, "ok": False, "error": "timeout"}
        print(json.dumps(res), flush=True)
        if res.get("rc", 0) < 0 or res.get("error") == "timeout":
            break  # a crashed / hung child: stop probing the GPU in this call


if __name__ == "__main__":
    main()
