"""Command-line flags.

The eight reference flags keep their names, defaults and absl/gflags syntax
(``--task_index=1`` or ``--task_index 1``; ``--sync``/``--nosync`` for bools):

    --ps_hosts ""  --worker_hosts ""  --job_name ""  --task_index 0
    --data_dir /data_dir  --model_dir /tmp/checkpoints  --workers 3  --ps 1

(``--ps`` is accepted and ignored, exactly as the reference never reads it.)
The reference's hard-coded hyper-parameters become flags whose defaults are
the reference values (per model), and the north-star additions are opt-in.
"""
from __future__ import annotations

import argparse


def _bool(v):
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("1", "true", "yes", "y", "t")


def add_bool(ap, name, default, help_):
    ap.add_argument("--" + name, dest=name, nargs="?", const=True, default=default, type=_bool, help=help_)
    ap.add_argument("--no" + name, dest=name, action="store_false", help=argparse.SUPPRESS)


# --heartbeat_secs default of --mode=allreduce: a survivor's watchdog aborts the collectives and exits
# non-zero --heartbeat_timeout seconds after a peer's last beat (parallel/health.py CommWatchdog)
AR_HEARTBEAT_SECS = 1.0


def resolve_mode(flags) -> str:
    """The run mode (explicit --mode, else ps when --ps_hosts is set, else allreduce when
    --worker_hosts is, else local) with the mode-dependent defaults filled in: --heartbeat_secs
    (None -> AR_HEARTBEAT_SECS for allreduce, 0 otherwise)."""
    mode = flags.mode or ("ps" if flags.ps_hosts else ("allreduce" if flags.worker_hosts else "local"))
    if flags.heartbeat_secs is None:
        flags.heartbeat_secs = AR_HEARTBEAT_SECS if mode == "allreduce" else 0.0
    return mode


def build_parser(model_defaults: dict | None = None, prog=None):
    d = dict(batch_size=None, num_steps=None, learning_rate=None)
    if model_defaults:
        d.update(model_defaults)
    ap = argparse.ArgumentParser(prog=prog, allow_abbrev=False)
    # ---- reference flags (GAN:31-45)
    ap.add_argument("--ps_hosts", default="", help="Comma-separated list of hostname:port pairs")
    ap.add_argument("--worker_hosts", default="", help="Comma-separated list of hostname:port pairs")
    ap.add_argument("--job_name", default="", help="One of 'ps', 'worker'")
    ap.add_argument("--task_index", type=int, default=0, help="Index of task within the job")
    ap.add_argument("--data_dir", default="/data_dir", help="Directory for storing mnist data")
    ap.add_argument("--model_dir", default="/tmp/checkpoints", help="Directory for storing the checkpoints")
    ap.add_argument("--workers", type=int, default=3, help="Number of workers")
    ap.add_argument("--ps", type=int, default=1, help="Number of ps (unused, as in the reference)")
    # ---- reference hyper-parameters as flags (defaults = C02 per model)
    ap.add_argument("--batch_size", type=int, default=d["batch_size"])
    ap.add_argument("--num_steps", type=int, default=d["num_steps"], help="global-step budget (training_steps)")
    ap.add_argument("--learning_rate", type=float, default=d["learning_rate"])
    # ---- lifecycle
    ap.add_argument("--save_model_secs", type=float, default=60.0)
    ap.add_argument("--save_summaries_secs", type=float, default=120.0)
    ap.add_argument("--max_to_keep", type=int, default=5)
    # ---- north-star / framework additions
    ap.add_argument("--mode", choices=["ps", "allreduce", "local"], default=None,
                    help="ps: between-graph parameter server (reference); allreduce: ring all-reduce DP; "
                         "local: single process. Default: ps when --ps_hosts is set, else allreduce/local")
    add_bool(ap, "sync", False, "sync SGD with a chief (SyncReplicasOptimizer semantics) in ps mode")
    ap.add_argument("--replicas_to_aggregate", type=int, default=None)
    ap.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto")
    ap.add_argument("--backend", choices=["auto", "gloo", "nccl"], default="auto")
    ap.add_argument("--seed", type=int, default=0)
    add_bool(ap, "hogwild", False, "lock-free ps updates (TF use_locking=False race)")
    add_bool(ap, "reinit_on_join", False, "every worker re-runs init (GAN:181 / ENC:160 quirk)")
    add_bool(ap, "py2_print", False, "print the Python-2 tuple form of the LSTM step line (LSTM:130)")
    add_bool(ap, "synthetic", False, "force synthetic MNIST-shaped data")
    add_bool(ap, "hip_graph", True, "capture the per-step kernels into a hipGraph (GPU)")
    ap.add_argument("--log_every", type=int, default=1, help="print the per-step line every N local steps")
    ap.add_argument("--comm_dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--bucket_mb", type=float, default=None,
                    help="all-reduce bucket size in MB of fp32 gradient (default: the model's own buckets - the "
                         "MNIST CNN's [head + fc1] / [convs] - else parallel/comm.py DEFAULT_BUCKET_MB); > 0")
    ap.add_argument("--dtype", choices=["auto", "fp32", "bf16"], default="auto",
                    help="compute dtype: fp32 = exact-fp32 MFMA kernels and fp32 activations (the reference's "
                         "precision), bf16 = bf16 MFMA with fp32 accumulation / masters; auto = the model's default. "
                         "GAN / autoencoder / LSTM / softmax: fp32 only; CNN: bf16 (default) or fp32; ResNets: bf16")
    ap.add_argument("--comm", choices=["auto", "rccl", "ipc", "pg"], default="auto",
                    help="all-reduce engine on GPUs: auto = faster of RCCL / hipIpc two-shot per bucket size "
                         "(both in-graph); pg = torch.distributed ProcessGroupNCCL (eager)")
    ap.add_argument("--ps_transport", choices=["auto", "native", "pg"], default="auto",
                    help="--mode=ps data plane: native = hipIpc mailboxes + C++ service thread (one node, GPUs; "
                         "parallel/ps_native.py), pg = torch.distributed send/recv; auto = native when eligible")
    ap.add_argument("--ps_partition_mb", type=float, default=0.0,
                    help="--mode=ps: split every variable larger than this many MB (fp32) into partitions "
                         "'<var>/part_<i>' dealt round-robin over the ps tasks (tf.variable_axis_size_partitioner "
                         "semantics; checkpoints keep the TF slice layout).  0: whole variables, as the reference")
    ap.add_argument("--metrics_jsonl", default="", help="append {step, gs, ms, images/sec, loss} lines here")
    ap.add_argument("--heartbeat_secs", type=float, default=None,
                    help="publish a TCPStore heartbeat every N s; 0: off.  Default: %s s in --mode=allreduce "
                         "(failure detection on: a dead peer ends every rank), 0 in --mode=ps / local (the "
                         "reference has no heartbeat)" % AR_HEARTBEAT_SECS)
    ap.add_argument("--heartbeat_timeout", type=float, default=30.0,
                    help="ps: count a worker silent for this long as lost; all-reduce: a rank whose peer "
                         "is silent this long aborts the collectives and exits non-zero (with --heartbeat_secs)")
    add_bool(ap, "phase_timers", False, "time fwd+bwd / comm / apply per step with hipEvents (no hipGraph)")
    add_bool(ap, "check_pull", False, "debug: checksum the pulled parameters every step (ps mode) / the "
                                      "replicas' parameters at the end (all-reduce mode)")
    ap.add_argument("--trace_json", default="", help="write the per-step phase timings as a Chrome trace "
                                                     "(chrome://tracing / Perfetto); implies --phase_timers")
    return ap


def parse(argv=None, model_defaults=None, prog=None):
    ap = build_parser(model_defaults, prog)
    args, unknown = ap.parse_known_args(argv)
    if unknown:
        ap.error("unknown flags: %s" % " ".join(unknown))
    return args
