"""T0: reference CLI parsing, cluster-spec rank map, round-robin placement."""
import pytest

from dtfe.models.autoencoder import AutoencoderModel
from dtfe.models.gan import GanModel
from dtfe.models.lstm import LstmModel
from dtfe.parallel.cluster import ClusterSpec
from dtfe.parallel.placement import device_string, round_robin, shard_vars
from dtfe.utils import flags


def test_reference_flag_defaults_and_absl_syntax():
    a = flags.parse([])
    assert (a.ps_hosts, a.worker_hosts, a.job_name, a.task_index) == ("", "", "", 0)
    assert (a.data_dir, a.model_dir, a.workers, a.ps) == ("/data_dir", "/tmp/checkpoints", 3, 1)
    a = flags.parse(["--ps_hosts=localhost:2222", "--worker_hosts", "localhost:2223,localhost:2224",
                     "--job_name=worker", "--task_index=1", "--workers=2", "--sync", "--nohogwild"])
    assert a.ps_hosts == "localhost:2222" and a.worker_hosts.endswith("2224")
    assert a.job_name == "worker" and a.task_index == 1 and a.workers == 2
    assert a.sync is True and a.hogwild is False
    assert flags.parse(["--sync=false"]).sync is False
    with pytest.raises(SystemExit):
        flags.parse(["--not_a_flag=1"])


def test_heartbeat_default_per_mode():
    """Failure detection is on by default in --mode=allreduce and off in --mode=ps / local (the
    reference has no heartbeat); an explicit value always wins."""
    a = flags.parse(["--worker_hosts=w0:1,w1:2"])
    assert a.heartbeat_secs is None
    assert flags.resolve_mode(a) == "allreduce" and a.heartbeat_secs == flags.AR_HEARTBEAT_SECS > 0
    a = flags.parse(["--ps_hosts=p:1", "--worker_hosts=w0:1"])
    assert flags.resolve_mode(a) == "ps" and a.heartbeat_secs == 0.0
    a = flags.parse([])
    assert flags.resolve_mode(a) == "local" and a.heartbeat_secs == 0.0
    a = flags.parse(["--worker_hosts=w0:1", "--heartbeat_secs=0"])
    assert flags.resolve_mode(a) == "allreduce" and a.heartbeat_secs == 0.0
    a = flags.parse(["--ps_hosts=p:1", "--mode=allreduce", "--heartbeat_secs=2.5"])
    assert flags.resolve_mode(a) == "allreduce" and a.heartbeat_secs == 2.5


def test_model_hyperparameter_defaults():
    a = flags.parse([], model_defaults=dict(batch_size=128, num_steps=100000, learning_rate=0.0002))
    assert (a.batch_size, a.num_steps, a.learning_rate) == (128, 100000, 0.0002)
    assert a.save_model_secs == 60.0 and a.max_to_keep == 5


def test_cluster_spec_rank_map():
    c = ClusterSpec.from_flags("h0:1,h1:2", "w0:3,w1:4,w2:5")
    assert c.world_size == 5
    assert c.rank_of("ps", 1) == 1 and c.rank_of("worker", 0) == 2 and c.rank_of("worker", 2) == 4
    assert c.task_of(3) == ("worker", 1)
    assert c.store_address() == ("h0", 1)
    assert ClusterSpec.from_flags("", "w0:9").store_address() == ("w0", 9)
    with pytest.raises(ValueError):
        c.rank_of("worker", 3)
    with pytest.raises(ValueError):
        c.rank_of("chief", 0)


def test_round_robin_placement_golden_gan_two_ps():
    g = GanModel()
    pl = round_robin(g.var_order, 2)
    # with 2 ps, W_genh1, W_disc1, b_genh1, b_disc1 and global_step on ps0
    assert shard_vars(pl, 0) == ["Variable", "Variable_2", "Variable_4", "Variable_6", "Variable_8"]
    assert shard_vars(pl, 1) == ["Variable_1", "Variable_3", "Variable_5", "Variable_7"]
    assert device_string(pl, "Variable_3", 0) == "/job:ps/task:1"


def test_round_robin_single_ps_and_lstm():
    assert set(round_robin(AutoencoderModel().var_order, 1).values()) == {0}
    pl = round_robin(LstmModel().var_order, 3)
    assert pl["rnn/basic_lstm_cell/kernel"] == 2 and pl["Variable_2"] == 1
