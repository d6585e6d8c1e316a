"""utils/graphs.py: several training steps per hipGraph replay (MultiStepGraph)."""
import pytest
import torch

from dtfe.utils.graphs import MultiStepGraph

pytestmark = pytest.mark.gpu


def test_multistep_graph_runs_exactly_n_steps():
    """run(n) executes exactly n steps - whole S-step replays, then single-step replays - and prime() captures
    both graphs up front (its steps are real steps too)."""
    x = torch.zeros(1, device="cuda")
    log = torch.zeros(64, device="cuda")

    def step():
        x.add_(1.0)
        log[x.long() % 64] += 1.0  # a second, state-dependent launch per step

    g = MultiStepGraph(step, 3, warmup=2)
    primed = g.prime()
    assert g.many.graph is not None and g.one.graph is not None
    torch.cuda.synchronize()
    assert int(x.item()) == primed
    for n in (7, 3, 1, 0, 5):
        before = int(x.item())
        g.run(n)
        torch.cuda.synchronize()
        assert int(x.item()) == before + n
    assert int(log.sum().item()) == int(x.item())


def test_multistep_cnn_steps_match_single_step_replays():
    """The MNIST-CNN trainer: 8 steps as two 4-step replays give the same parameters, bitwise, as 8
    single-step replays from the same state (same device-side sampling and dropout counters)."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer
    out = []
    for S in (1, 4):
        tr = MnistCnnTrainer(256, "cuda:0", seed=0)
        g = MultiStepGraph(tr.step, S, warmup=2)
        g.run(8)
        torch.cuda.synchronize()
        out.append((tr.P.master.clone(), int(tr.global_step.item())))
    assert out[0][1] == out[1][1] == 8
    assert torch.equal(out[0][0], out[1][0])


def test_deferred_join_cnn_matches_joined_steps():
    """MnistCnnTrainer.defer_join (bench.py, several steps per replay): the conv2 weight-gradient branch
    signals Adam through a device counter and rejoins once per replay - 8 steps as two 4-step replays give
    the joined-every-step parameters bitwise, eagerly and replayed."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer
    out = []
    for defer, graph in ((False, True), (True, True), (True, False)):
        tr = MnistCnnTrainer(256, "cuda:0", seed=0)
        tr.defer_join = defer
        g = MultiStepGraph(tr.step, 4, warmup=2, enabled=graph, finish=tr.join_side)
        g.run(8)  # (graph: the first 4-step block eager, the second captured and replayed)
        torch.cuda.synchronize()
        out.append((tr.P.master.clone(), int(tr.global_step.item()), int(tr.c2_done.item()), int(tr.c2_seen.item())))
    ref = out[0]
    for m, gs, done, seen in out[1:]:
        assert torch.equal(m, ref[0])
        assert done == seen == gs  # one signal and one consume per step
    assert ref[2] == ref[3] == 0
