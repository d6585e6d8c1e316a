"""T1/T2: multi-process clusters on 127.0.0.1 with the exact reference CLI (gloo, CPU).

BASELINE.json config 1 (softmax regression, 1 ps + 2 workers, async SGD on
CPU/gloo) plus the reference lifecycle: done protocol, chief-only
checkpoints, global step budget, restore-on-restart, sync mode, 2 ps shards,
all-reduce mode and a killed non-chief worker.
"""
import os
import re
import subprocess
import sys
import time

import pytest
import torch

from dtfe import ckpt

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "launch"))
import local_cluster  # noqa: E402

pytestmark = pytest.mark.slow
COMMON = ["--data_dir=/nonexistent", "--device=cpu", "--seed=1"]


def _gs_lines(lines):
    return [int(m.group(1)) for l in lines for m in [re.match(r"Global step (\d+) Local step \d+  AvgTime: [\d.]+ms", l)]
            if m]


def test_softmax_1ps_2workers_async(tmp_path):
    md = str(tmp_path / "ck")
    codes, out, _ = local_cluster.launch("softmax", 1, 2, COMMON + ["--num_steps=60", "--workers=2",
                                                                     "--model_dir=" + md, "--save_model_secs=0.2"],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), (codes, out)
    ps = out[("ps", 0)]
    assert "ps 0 received done 0" in ps and "ps 0 received done 1" in ps
    assert ps[-1] == "ps 0: quitting"
    for w in (0, 1):
        assert any(l.startswith("Total Time: ") for l in out[("worker", w)])
    gs = _gs_lines(out[("worker", 0)]) + _gs_lines(out[("worker", 1)])
    assert max(gs) >= 60 and max(gs) <= 61  # async total ~N (<= 1 extra step per worker)
    # chief-only checkpoints, TF layout
    latest = ckpt.latest_checkpoint(md)
    assert latest is not None
    t = ckpt.load_bundle(latest)
    assert set(t) == {"Variable", "Variable_1", "Variable_2"} and t["Variable"].shape == (784, 10)
    assert os.path.exists(os.path.join(md, "graph.pbtxt"))
    assert any(f.startswith("events.out.tfevents.") for f in os.listdir(md))


def test_chief_restart_restores_global_step(tmp_path):
    md = str(tmp_path / "ck")
    args = COMMON + ["--workers=1", "--model_dir=" + md, "--save_model_secs=0.05"]
    codes, out, _ = local_cluster.launch("softmax", 1, 1, args + ["--num_steps=40"], timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    saved = int(ckpt.load_bundle(ckpt.latest_checkpoint(md))["Variable_2"])
    assert saved > 0
    codes, out, _ = local_cluster.launch("softmax", 1, 1, args + ["--num_steps=%d" % (saved + 10)], timeout=240,
                                         stream=False)
    assert all(c == 0 for c in codes.values()), (codes, {k: v[-12:] for k, v in out.items()})
    gs = _gs_lines(out[("worker", 0)])
    assert gs[0] == saved + 1, (saved, gs[:3])  # resumed, not re-initialised (LSTM-style correct resume)


def test_reinit_on_join_quirk(tmp_path):
    md = str(tmp_path / "ck")
    args = COMMON + ["--workers=1", "--model_dir=" + md, "--save_model_secs=0.05"]
    local_cluster.launch("softmax", 1, 1, args + ["--num_steps=30"], timeout=240, stream=False)
    codes, out, _ = local_cluster.launch("softmax", 1, 1, args + ["--num_steps=10", "--reinit_on_join"],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), (codes, {k: v[-15:] for k, v in out.items()})
    # GAN:181 / ENC:160 behaviour: the re-init clobbers the restored step counter
    assert _gs_lines(out[("worker", 0)])[0] == 1


def test_two_ps_shards_and_lstm_eval(tmp_path):
    md = str(tmp_path / "ck")
    codes, out, _ = local_cluster.launch("lstm", 2, 2, COMMON + ["--num_steps=6", "--workers=2", "--batch_size=128",
                                                                  "--model_dir=" + md, "--save_model_secs=0.3"],
                                         timeout=300, stream=False)
    assert all(c == 0 for c in codes.values()), out
    for p in (0, 1):
        assert out[("ps", p)][-1] == "ps %d: quitting" % p
    for w in (0, 1):
        assert any(re.match(r"Test-Accuracy: \d\.\d{4}$", l) for l in out[("worker", w)])
    t = ckpt.load_bundle(ckpt.latest_checkpoint(md))
    assert t["rnn/basic_lstm_cell/kernel"].shape == (156, 512)
    assert t["Variable_2"].dtype == torch.int32


def test_sync_mode_steps_in_lockstep(tmp_path):
    codes, out, _ = local_cluster.launch("softmax", 1, 2, COMMON + ["--num_steps=20", "--workers=2", "--sync",
                                                                     "--save_model_secs=0",
                                                                     "--model_dir=" + str(tmp_path)],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    g0, g1 = _gs_lines(out[("worker", 0)]), _gs_lines(out[("worker", 1)])
    # every global step aggregates both replicas: each worker sees consecutive steps 1, 2, 3 ...
    assert g0[:5] == [1, 2, 3, 4, 5] and g1[:5] == [1, 2, 3, 4, 5]


def test_gan_global_step_advances_by_two(tmp_path):
    codes, out, _ = local_cluster.launch("gan", 1, 1, COMMON + ["--num_steps=10", "--workers=1",
                                                                 "--save_model_secs=0", "--batch_size=16",
                                                                 "--model_dir=" + str(tmp_path)],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    assert _gs_lines(out[("worker", 0)])[:3] == [2, 4, 6]


def test_allreduce_mode_two_workers(tmp_path):
    codes, out, _ = local_cluster.launch("encoder", 0, 2, COMMON + ["--num_steps=5", "--mode=allreduce",
                                                                     "--batch_size=32", "--save_model_secs=0",
                                                                     "--model_dir=" + str(tmp_path)],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    assert _gs_lines(out[("worker", 0)]) == [1, 2, 3, 4, 5]
    assert _gs_lines(out[("worker", 1)]) == [1, 2, 3, 4, 5]


def test_allreduce_rank_crash_ends_every_rank_cpu(tmp_path):
    """--mode=allreduce with default flags (no --heartbeat_secs): worker 1 crashes at step 5, worker
    0 must not hang - its comm watchdog (on by default in this mode) or the gloo collective ends it
    with a non-zero code."""
    env = dict(os.environ, DTFE_FAULT="crash@worker:1:step=5")
    t0 = time.time()
    codes, out, _ = local_cluster.launch("encoder", 0, 2, COMMON + [
        "--num_steps=100000", "--mode=allreduce", "--batch_size=32", "--save_model_secs=0",
        "--heartbeat_timeout=3", "--model_dir=" + str(tmp_path)], env=env, timeout=200, stream=False)
    assert time.time() - t0 < 150
    assert codes[("worker", 1)] == 17, out[("worker", 1)][-10:]
    assert codes[("worker", 0)] not in (0, None), (codes, out[("worker", 0)][-20:])


def test_killed_non_chief_worker_does_not_stall_others(tmp_path):
    """device_filters semantics: worker 1 dies, worker 0 finishes; the ps keeps waiting
    for the missing done signal exactly like the reference (C07) until we stop it."""
    ports = local_cluster.free_ports(3)
    ps_hosts = "127.0.0.1:%d" % ports[0]
    wh = "127.0.0.1:%d,127.0.0.1:%d" % (ports[1], ports[2])
    base = COMMON + ["--workers=2", "--save_model_secs=0", "--model_dir=" + str(tmp_path)]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    mk = lambda job, i, extra: subprocess.Popen(local_cluster.task_argv("softmax", ps_hosts, wh, job, i, base + extra),
                                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    ps = mk("ps", 0, ["--num_steps=400"])
    w0 = mk("worker", 0, ["--num_steps=400"])
    w1 = mk("worker", 1, ["--num_steps=100000"])
    try:
        time.sleep(8)
        w1.kill()
        out0, _ = w0.communicate(timeout=180)
        assert w0.returncode == 0, out0
        assert "Total Time" in out0
        time.sleep(1)
        assert ps.poll() is None  # still waiting for worker 1's done signal
    finally:
        for p in (ps, w0, w1):
            if p.poll() is None:
                p.kill()


def test_cnn_1ps_2workers_async_checkpoint_keys(tmp_path):
    """BASELINE.json config 4 on CPU/gloo: the MNIST CNN through the ps roles, TF variable names
    (Variable..Variable_7 + Adam slots + beta powers + global step Variable_8) in the checkpoint."""
    md = str(tmp_path / "ck")
    codes, out, _ = local_cluster.launch("cnn", 1, 2, COMMON + ["--num_steps=6", "--workers=2", "--batch_size=8",
                                                                 "--model_dir=" + md, "--save_model_secs=0.1"],
                                         timeout=300, stream=False)
    assert all(c == 0 for c in codes.values()), (codes, out)
    steps = _gs_lines(out[("worker", 0)]) + _gs_lines(out[("worker", 1)])
    assert max(steps) >= 6
    t = ckpt.load_bundle(ckpt.latest_checkpoint(md))
    assert tuple(t["Variable"].shape) == (5, 5, 1, 32)          # TF layout [KH][KW][Cin][Cout]
    assert tuple(t["Variable_2"].shape) == (3136, 1024)         # fc1 [in][out]
    assert "Variable_2/Adam" in t and "Variable_2/Adam_1" in t and "beta1_power" in t
    assert int(t["Variable_8"]) >= 1


def test_fault_injection_crash_with_heartbeat_lets_ps_quit(tmp_path):
    """DTFE_FAULT crashes worker 1 at step 5 (no done signal, like a killed pod); with heartbeats
    the ps counts it lost after the timeout and still quits, while worker 0 finishes normally."""
    env = dict(os.environ, DTFE_FAULT="crash@worker:1:step=5")
    codes, out, _ = local_cluster.launch("softmax", 1, 2, COMMON + [
        "--num_steps=300", "--workers=2", "--model_dir=" + str(tmp_path / "ck"), "--save_model_secs=0",
        "--heartbeat_secs=0.2", "--heartbeat_timeout=2"], env=env, timeout=240, stream=False)
    assert codes[("worker", 1)] == 17, out[("worker", 1)]
    assert any("fault injection: worker 1 crashes" in l for l in out[("worker", 1)])
    assert codes[("worker", 0)] == 0 and any(l.startswith("Total Time") for l in out[("worker", 0)])
    ps = out[("ps", 0)]
    assert codes[("ps", 0)] == 0, ps
    assert any("ps 0: worker 1 lost" in l for l in ps) and ps[-1] == "ps 0: quitting"


def test_phase_timers_and_check_pull(tmp_path):
    codes, out, _ = local_cluster.launch("softmax", 1, 1, COMMON + [
        "--num_steps=3", "--workers=1", "--model_dir=" + str(tmp_path / "ck"), "--save_model_secs=0",
        "--check_pull"], timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    assert any(l.startswith("pull checksum gs=") for l in out[("worker", 0)])


def test_chrome_trace_of_phases(tmp_path):
    import json
    tr = str(tmp_path / "trace.json")
    codes, out, _ = local_cluster.launch("encoder", 0, 1, COMMON + [
        "--mode=local", "--num_steps=3", "--model_dir=" + str(tmp_path / "ck"), "--save_model_secs=0",
        "--batch_size=16", "--trace_json=" + tr], timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    ev = json.load(open(tr))["traceEvents"]
    assert {e["name"] for e in ev} >= {"fwd+bwd", "apply"} and all(e["ph"] == "X" and e["dur"] >= 0 for e in ev)
    assert len([e for e in ev if e["name"] == "apply"]) == 3


def test_killed_ps_makes_workers_error_out(tmp_path):
    """when the ps dies, workers error out on their next exchange and exit
    non-zero (no hang); the reference gives the same outcome through failing RecvTensor RPCs."""
    env = dict(os.environ, DTFE_FAULT="crash@ps:0:step=10")
    codes, out, _ = local_cluster.launch("softmax", 1, 2, COMMON + [
        "--num_steps=100000", "--workers=2", "--model_dir=" + str(tmp_path / "ck"), "--save_model_secs=0"],
        env=env, timeout=240, stream=False)
    assert codes[("ps", 0)] == 17, out[("ps", 0)]
    assert any("fault injection: ps 0 crashes" in l for l in out[("ps", 0)])
    for w in (0, 1):
        assert codes[("worker", w)] != 0, out[("worker", w)][-5:]
        assert not any(l.startswith("Total Time") for l in out[("worker", w)])


def test_sync_three_workers_two_replicas_terminates(tmp_path):
    """--replicas_to_aggregate below the worker count: the last round may be left with fewer
    fresh gradients than R once workers finish; the ps must release it and the job must end."""
    codes, out, _ = local_cluster.launch("softmax", 1, 3, COMMON + ["--num_steps=15", "--workers=3", "--sync",
                                                                     "--replicas_to_aggregate=2",
                                                                     "--save_model_secs=0",
                                                                     "--model_dir=" + str(tmp_path)],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), {k: v[-15:] for k, v in out.items()}
    assert "ps 0: quitting" in out[("ps", 0)]
    assert max(max(_gs_lines(out[("worker", w)]) or [0]) for w in range(3)) >= 15


def test_lstm_non_default_batch_evaluates(tmp_path):
    """Test-Accuracy over the reference's 128 test images with a 64-image program batch."""
    codes, out, _ = local_cluster.launch("lstm", 1, 1, COMMON + ["--num_steps=3", "--workers=1", "--batch_size=64",
                                                                  "--save_model_secs=0", "--model_dir=" + str(tmp_path)],
                                         timeout=240, stream=False)
    assert all(c == 0 for c in codes.values()), out
    assert any(re.match(r"Test-Accuracy: \d\.\d{4}$", l) for l in out[("worker", 0)])
    assert "ps 0: quitting" in out[("ps", 0)]


def test_shard_apply_takes_the_payload_not_a_shared_buffer():
    """Hogwild applies run without the shard lock: each one must read its own payload (never a
    gradient staged in the shard's shared P.grad, which a concurrent push could overwrite)."""
    import threading

    from dtfe.models.softmax_reg import SoftmaxRegressionModel
    from dtfe.parallel.ps import Shard

    m = SoftmaxRegressionModel()
    specs = [s for s in m.specs]
    sh = Shard(specs, m.opt_groups, "cpu", True, m.gs_increments)
    sh.P.master.zero_()
    sh.P.refresh_copies()
    sh.P.grad.fill_(float("nan"))            # anything read from here would poison the params
    lr = m.opt_groups[0][0].lr
    ga = torch.full((sh.P.total,), 1.0)
    gb = torch.full((sh.P.total,), 2.0)
    ths = [threading.Thread(target=lambda g=g: [sh.apply(g) for _ in range(5)]) for g in (ga, gb)]
    for t in ths:  # one after the other: lock-free applies may legitimately race on the params
        t.start()
        t.join()
    v = sh.P.view(specs[0].name)
    assert torch.isfinite(v).all()
    assert torch.allclose(v, torch.full_like(v, -lr * 15.0), rtol=1e-5)
    assert sh.global_step() == 10
