"""ConsensusEngine.step_pipelined (update scatter of one instance range overlapped with the round of
the previous range on HIP streams) == apply_updates(unique=True) + run_round, bit for bit, eager and
inside a captured HIP graph."""
import pytest
import torch

from svoc.config import ConsensusConfig
from svoc.engine import ConsensusEngine
from svoc.stream import SyntheticUpdateStream

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIELDS = ("values", "enabled", "n_active", "touched", "consensus_active", "c1", "consensus", "skew", "kurt",
          "rel", "qr", "reliable", "status", "metrics_fx")


def _pair(N, D, f, B, constrained=True):
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=constrained)
    a = ConsensusEngine(cfg, batch=B, device=DEV)
    b = ConsensusEngine(cfg, batch=B, device=DEV)
    a.randomize(seed=3)
    b.randomize(seed=3)
    return a, b


def _same(a, b):
    torch.cuda.synchronize()
    for k in FIELDS:
        torch.testing.assert_close(getattr(a, k), getattr(b, k), rtol=0, atol=0, equal_nan=True, msg=k)


@pytest.mark.parametrize("N,D,f,B,U,chunks", [(256, 512, 32, 10, 64, 2), (256, 300, 32, 7, 16, 3),
                                               (64, 1024, 8, 9, 8, 4), (7, 6, 2, 33, 1, 2),
                                               (128, 200, 40, 6, 32, 2)])
def test_step_pipelined_matches_serial(N, D, f, B, U, chunks):
    a, b = _pair(N, D, f, B)
    st = SyntheticUpdateStream(B, N, D, U, f, pool=2, device=DEV, seed=5)
    for i in range(3):
        inst, orc, vals = st.batch(i)
        a.step_pipelined(inst, orc, vals, U, chunks=chunks)
        b.apply_updates(inst, orc, vals, unique=True)
        b.run_round()
        _same(a, b)


def test_step_pipelined_in_graph():
    N, D, f, B, U = 256, 640, 32, 8, 64
    a, b = _pair(N, D, f, B)
    st = SyntheticUpdateStream(B, N, D, U, f, pool=2, device=DEV, seed=9)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture (allocations, stream creation)
        a.step_pipelined(*st.batch(0), U, chunks=2)
    torch.cuda.current_stream().wait_stream(s)
    b.apply_updates(*st.batch(0), unique=True)
    b.run_round()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        a.step_pipelined(*st.batch(1), U, chunks=2)
    for _ in range(2):
        g.replay()
        b.apply_updates(*st.batch(1), unique=True)
        b.run_round()
    _same(a, b)


def test_step_pipelined_rejects_ungrouped_batch():
    a, _ = _pair(64, 128, 8, 4)
    with pytest.raises(ValueError):
        a.step_pipelined(torch.zeros(3, dtype=torch.long, device=DEV), torch.zeros(3, dtype=torch.long, device=DEV),
                         torch.zeros(3, 128, device=DEV), 2, chunks=2)


@pytest.mark.parametrize("chunks", [2, 3])
def test_step_pipelined_overlap_matches_serial(chunks):
    """overlap=True: consecutive steps overlap (range 0's update beside the previous step's last round;
    each range's update waits only for the previous step's round of that range) -- same state."""
    N, D, f, B, U = 256, 512, 32, 9, 64
    a, b = _pair(N, D, f, B)
    st = SyntheticUpdateStream(B, N, D, U, f, pool=2, device=DEV, seed=7)
    for i in range(4):
        a.step_pipelined(*st.batch(i), U, chunks=chunks, overlap=True)
        b.apply_updates(*st.batch(i), unique=True)
        b.run_round()
    m = a.metrics()            # joins the open pipeline before reading
    assert not a._pipe_open
    _same(a, b)
    assert torch.equal(m, b.metrics())


def test_step_pipelined_overlap_in_graph():
    """Four overlapped steps captured in one graph (joined at the end of the capture), replayed twice."""
    N, D, f, B, U = 256, 640, 32, 8, 64
    a, b = _pair(N, D, f, B)
    st = SyntheticUpdateStream(B, N, D, U, f, pool=2, device=DEV, seed=11)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture (allocations, stream creation)
        a.step_pipelined(*st.batch(0), U, chunks=2, overlap=True)
        a.pipeline_join()
    torch.cuda.current_stream().wait_stream(s)
    b.apply_updates(*st.batch(0), unique=True)
    b.run_round()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(4):
            a.step_pipelined(*st.batch(i + 1), U, chunks=2, overlap=True)
        a.pipeline_join()
    for _ in range(2):
        g.replay()
        for i in range(4):
            b.apply_updates(*st.batch(i + 1), unique=True)
            b.run_round()
    _same(a, b)
