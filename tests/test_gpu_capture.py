"""engine.capture_guard against the capture topology that segfaults hipStreamEndCapture on this
HIP stack (tools/capture_probe.py `pingpong`, profiles/r6_capture_bisect.log): two side streams
of a capture waiting on each other in turn.  The guard refuses the second wait with
CaptureTopologyError before it is made (the process survives and can capture again), and leaves
the origin <-> side-stream alternation the bench's pipelined lanes use alone."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_capture_guard_refuses_side_stream_pingpong():
    from bikg_graph_explainability_public_amd import engine
    x = torch.ones(1 << 12, device=DEV)
    a, b = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(engine.CaptureTopologyError):
        with engine.capture_guard(), torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            a.wait_stream(cur)
            b.wait_stream(cur)
            with torch.cuda.stream(a):
                x.add_(1.0)
            b.wait_stream(a)
            with torch.cuda.stream(b):
                x.mul_(2.0)
            a.wait_stream(b)  # refused: b waited on a
    torch.cuda.synchronize()
    # the stream methods are restored and the process captures again
    assert torch.cuda.Stream.wait_stream.__name__ == "wait_stream"
    g2 = torch.cuda.CUDAGraph()
    y = torch.ones(1 << 12, device=DEV)
    with engine.capture_guard(), torch.cuda.graph(g2):
        y.mul_(3.0)
    g2.replay()
    torch.cuda.synchronize()
    assert float(y[0]) == 3.0


def test_capture_guard_allows_origin_side_alternation():
    from bikg_graph_explainability_public_amd import engine
    x = torch.zeros(1 << 12, device=DEV)
    s1 = torch.cuda.Stream(device=DEV)
    ev = torch.cuda.Event()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with engine.capture_guard(), torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        for _ in range(4):  # the bench's pipe_step pattern: s1 <- cur, s1 work, cur <- s1 (event)
            s1.wait_stream(cur)
            with torch.cuda.stream(s1):
                x.add_(1.0)
                ev.record(s1)
                s1.wait_stream(cur)
                x.mul_(2.0)
            cur.wait_event(ev)
        cur.wait_stream(s1)
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 30.0  # ((((0+1)*2+1)*2+1)*2+1)*2
