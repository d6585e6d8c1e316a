"""Variable -> ps shard placement.

``tf.train.replica_device_setter(cluster=...)`` (GAN:119-121) places the k-th
*created* variable on ``/job:ps/task:(k mod P)`` (round-robin ``ps_strategy``);
optimizer slots and Adam's beta powers are colocated with their primary
variable and do not advance k.  ``global_step`` is a variable like any other
and takes its creation ordinal.
"""
from __future__ import annotations


def round_robin(var_names_in_creation_order, num_ps: int) -> dict:
    """{var name: ps task index}."""
    if num_ps <= 0:
        return {n: None for n in var_names_in_creation_order}
    return {n: k % num_ps for k, n in enumerate(var_names_in_creation_order)}


def shard_vars(placement: dict, ps_task: int):
    return [n for n, t in placement.items() if t == ps_task]


def device_string(placement: dict, name: str, worker_task: int) -> str:
    """The TF device string the reference would assign (for logging / graph.pbtxt)."""
    t = placement.get(name)
    if t is None:
        return "/job:worker/task:%d" % worker_task
    return "/job:ps/task:%d" % t
