"""Which graph-capture mistake ends capture_end in a segfault on this HIP stack (VERDICT r2 item 6:
`gpurun_out/pipe_dbg.log`, bench.py's pipelined capture at 04:56, Fatal Python error in
torch/cuda/graphs.py capture_end).

Each variant runs in its own child process (a crash ends only that child); the parent prints
one line per variant and stops at the first child killed by a signal:

  joined      side stream forked from the capture stream, work on it, joined back (control)
  sync        a host sync (.item()) inside the capture
  alloc_side  an allocation on a side stream that was never forked from the capture stream
  unjoined    side stream forked from the capture stream, work on it, NOT joined before the
              capture ends
  timing_ev   a timing-enabled CUDA event recorded inside the capture
  ext_wait    a side stream waits on an event recorded BEFORE the capture, then joins
  replay_in   another graph replayed while this one is being captured
  graph_gc    a graph object dropped (freed) while another is being captured

    python tools/capture_probe.py [variant ...]
"""
import subprocess
import sys

VARIANTS = ("joined", "sync", "alloc_side", "unjoined", "timing_ev", "ext_wait", "replay_in",
            "graph_gc")


def child(variant):
    import torch
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 20, device=dev)
    side = torch.cuda.Stream(device=dev)
    pre = torch.cuda.Event()
    pre.record()
    other = torch.cuda.CUDAGraph()
    if variant in ("replay_in", "graph_gc"):
        with torch.cuda.graph(other):
            x.mul_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        y = x * 2
        if variant == "timing_ev":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        elif variant == "ext_wait":
            side.wait_event(pre)
            with torch.cuda.stream(side):
                z = x + 1
            cur.wait_stream(side)
        elif variant == "replay_in":
            other.replay()
        elif variant == "graph_gc":
            del other
            import gc
            gc.collect()
        elif variant == "sync":
            float(y.sum().item())
        elif variant == "alloc_side":
            with torch.cuda.stream(side):  # never waited on the capture stream
                z = torch.empty(1 << 20, device=dev)
                z.fill_(3.0)
        else:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                y.add_(1.0)
            if variant == "joined":
                cur.wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    print(f"{variant}: capture + replay ok, y[0] = {float(y[0])}", flush=True)


def main():
    wanted = sys.argv[1:] or list(VARIANTS)
    for v in wanted:
        p = subprocess.run([sys.executable, __file__, "--child", v], capture_output=True, text=True,
                           timeout=300)
        tail = (p.stdout + p.stderr).strip().splitlines()
        msg = [t for t in tail if "Error" in t or "error" in t or "ok" in t][-2:]
        print(f"[capture_probe] {v}: exit {p.returncode} | {' | '.join(msg)[:400]}", flush=True)
        if p.returncode < 0 or p.returncode in (134, 139):
            print("[capture_probe] child killed by a signal: stopping", flush=True)
            return 0
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        sys.exit(main())
