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
  multi_side  four side streams forked from the capture stream, work on each, all joined
  xstream_ev  side stream A records an event after its work, side stream B waits for it, then
              works; both joined
  ev_rerecord one event recorded twice on A (after two pieces of work), waited by B after the
              first record and by C after the second; all joined
  ev_dangling an event recorded on a joined side stream that nothing waits for
  pipe2       bench.py's fit-depth-2 pipelined topology with torch ops standing in for the
              kernels: two graphs of 4 steps, 4 buffer sets, two fit streams, a production and a
              finish stream, per-set events waited only inside their own capture
  pipe2_fresh pipe2 with new event objects for each capture (no event recorded in two captures)

    python tools/capture_probe.py [variant ...]
"""
import subprocess
import sys

VARIANTS = ("joined", "sync", "alloc_side", "unjoined", "timing_ev", "ext_wait", "replay_in",
            "graph_gc", "multi_side", "xstream_ev", "ev_rerecord", "ev_dangling", "pipe2_fresh", "pipe2")


def pipe2(fresh=False, graphs_n=2, ev_prod=True, ev_fin=True, ev_fit=True, unroll=4):
    import torch
    dev = torch.device("cuda", 0)
    n_sets = 4
    sets = [torch.zeros(1 << 16, device=dev) for _ in range(n_sets)]
    res = [torch.zeros(1 << 16, device=dev) for _ in range(n_sets)]
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    fs = [torch.cuda.Stream(device=dev) for _ in range(2)]
    prod = [torch.cuda.Event() for _ in range(n_sets)]
    fit = [torch.cuda.Event() for _ in range(n_sets)]
    fin = [torch.cuda.Event() for _ in range(n_sets)]
    sets[0].fill_(1.0)
    torch.cuda.synchronize()
    graphs = []
    for b in range(graphs_n):
        g = torch.cuda.CUDAGraph()
        if fresh:  # event objects of this capture only (none re-recorded in another capture)
            prod = [torch.cuda.Event() for _ in range(n_sets)]
            fit = [torch.cuda.Event() for _ in range(n_sets)]
            fin = [torch.cuda.Event() for _ in range(n_sets)]
        with torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            for st in (s1, s2, *fs):
                st.wait_stream(cur)
            rec = set()
            for j in range(unroll):
                i = b * unroll + j
                a, nb = i % n_sets, (i + 1) % n_sets
                f = fs[i & 1]
                if ("prod", a) in rec:
                    f.wait_event(prod[a])
                elif not ev_prod and j > 0:
                    f.wait_stream(s1)
                with torch.cuda.stream(f):
                    res[a].copy_(sets[a] * 2.0)
                    if ev_fit:
                        fit[a].record(f)
                with torch.cuda.stream(s1):
                    if ("fin", nb) in rec:
                        s1.wait_event(fin[nb])
                    elif not ev_fin:
                        s1.wait_stream(s2)
                    sets[nb].fill_(float(i + 2))
                    if ev_prod and j + 1 < unroll:
                        prod[nb].record(s1)
                        rec.add(("prod", nb))
                if ev_fit:
                    s2.wait_event(fit[a])
                else:
                    s2.wait_stream(f)
                with torch.cuda.stream(s2):
                    res[a].add_(0.5)
                    if ev_fin and j + n_sets - 1 < unroll:
                        fin[a].record(s2)
                        rec.add(("fin", a))
            for st in (s1, s2, *fs):
                cur.wait_stream(st)
        graphs.append(g)
    for m in range(4):
        graphs[m % graphs_n].replay()
    torch.cuda.synchronize()
    print(f"pipe2 (fresh={fresh} graphs={graphs_n} ev prod/fin/fit={ev_prod}/{ev_fin}/{ev_fit} u={unroll}): capture + replay ok, res[3][0] = {float(res[3][0])}", flush=True)


def chain(kind):
    """Minimal wait_stream constructs among side streams forked from the capture stream (round-6
    bisection of the pipe2 segfault), each joined back before the capture ends:
      wait_empty   B waits A, A has no work since the fork; B works
      wait_chain   C waits B waits A, none of them worked yet; C works
      seq3         A works; B waits A, works; C waits B, works
      pingpong     A works; B waits A, works; A waits B, works
      ring3x2      two rounds of: A waits C, works; B waits A, works; C waits B, works
      ring3_first  ring3x2's first round only (A's first wait is on C before C worked)
      ring3_late   like ring3x2 but A's first wait skipped (every wait follows work)"""
    import torch
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 16, device=dev)
    ss = [torch.cuda.Stream(device=dev) for _ in range(3)]
    A, B, C = ss
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        for st in ss:
            st.wait_stream(cur)

        def work(st, v):
            with torch.cuda.stream(st):
                x.add_(v)
        if kind == "wait_empty":
            B.wait_stream(A)
            work(B, 1.0)
        elif kind == "wait_chain":
            B.wait_stream(A)
            C.wait_stream(B)
            work(C, 1.0)
        elif kind == "seq3":
            work(A, 1.0)
            B.wait_stream(A)
            work(B, 1.0)
            C.wait_stream(B)
            work(C, 1.0)
        elif kind == "pingpong":
            work(A, 1.0)
            B.wait_stream(A)
            work(B, 1.0)
            A.wait_stream(B)
            work(A, 1.0)
        elif kind == "pingpong_cur":  # the same alternation with the capture stream itself
            work(cur, 1.0)
            A.wait_stream(cur)
            work(A, 1.0)
            cur.wait_stream(A)
            work(cur, 1.0)
        elif kind == "pingpong_nowork_b":  # B forwards A's dependency without work of its own
            work(A, 1.0)
            B.wait_stream(A)
            A.wait_stream(B)
            work(A, 1.0)
        elif kind == "pingpong_end":  # A's second wait is its last operation
            work(A, 1.0)
            B.wait_stream(A)
            work(B, 1.0)
            A.wait_stream(B)
        elif kind == "pingpong_join_first":  # B joined to cur before A waits on B
            work(A, 1.0)
            B.wait_stream(A)
            work(B, 1.0)
            cur.wait_stream(B)
            A.wait_stream(cur)
            work(A, 1.0)
        else:
            rounds = 1 if kind == "ring3_first" else 2
            for r in range(rounds):
                if not (kind == "ring3_late" and r == 0):
                    A.wait_stream(C)
                work(A, 1.0)
                B.wait_stream(A)
                work(B, 1.0)
                C.wait_stream(B)
                work(C, 1.0)
        for st in ss:
            cur.wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    print(f"{kind}: capture + replay ok, x[0] = {float(x[0])}", flush=True)


CHAINS = ("wait_empty", "wait_chain", "seq3", "pingpong", "ring3_late", "ring3_first", "ring3x2",
          "pingpong_cur", "pingpong_nowork_b", "pingpong_end", "pingpong_join_first")


def child(variant):
    import torch
    if variant in CHAINS:
        return chain(variant)
    if variant in ("pipe2", "pipe2_fresh"):
        return pipe2(fresh=variant == "pipe2_fresh")
    if variant.startswith("p2:"):  # p2:g=1,prod=0,fin=1,fit=1,u=4
        kv = dict(x.split("=") for x in variant[3:].split(","))
        return pipe2(graphs_n=int(kv.get("g", 2)), ev_prod=kv.get("prod", "1") == "1",
                     ev_fin=kv.get("fin", "1") == "1", ev_fit=kv.get("fit", "1") == "1",
                     unroll=int(kv.get("u", 4)))
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
        elif variant in ("multi_side", "xstream_ev", "ev_rerecord", "ev_dangling"):
            ss = [torch.cuda.Stream(device=dev) for _ in range(4)]
            for st in ss:
                st.wait_stream(cur)
            ev = torch.cuda.Event()
            if variant == "multi_side":
                for k, st in enumerate(ss):
                    with torch.cuda.stream(st):
                        y[k::4].add_(1.0)
            elif variant == "xstream_ev":
                with torch.cuda.stream(ss[0]):
                    y.add_(1.0)
                    ev.record(ss[0])
                ss[1].wait_event(ev)
                with torch.cuda.stream(ss[1]):
                    y.mul_(2.0)
            elif variant == "ev_rerecord":
                with torch.cuda.stream(ss[0]):
                    y.add_(1.0)
                    ev.record(ss[0])
                ss[1].wait_event(ev)
                with torch.cuda.stream(ss[1]):
                    x.add_(0.0)
                with torch.cuda.stream(ss[0]):
                    y.add_(1.0)
                    ev.record(ss[0])
                ss[2].wait_event(ev)
                with torch.cuda.stream(ss[2]):
                    y.mul_(1.0)
            else:
                with torch.cuda.stream(ss[0]):
                    y.add_(1.0)
                    ev.record(ss[0])
            for st in ss:
                cur.wait_stream(st)
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
