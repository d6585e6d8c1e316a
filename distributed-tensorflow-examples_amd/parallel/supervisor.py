"""Chief-based lifecycle - ``tf.train.Supervisor`` equivalent.

Chief (``is_chief``, task 0):
  * ``prepare()``: restore from the latest checkpoint in ``logdir`` if one
    exists, else run the init function (push initial values to the ps shards);
    write ``graph.pbtxt`` + an events file with the variable graph;
  * checkpoint thread: save immediately, then every ``save_model_secs``, to
    ``logdir/model.ckpt-<global_step>`` (max_to_keep retention);
  * step-counter thread: every ``save_summaries_secs`` append
    ``global_step/sec`` to the events file.
Non-chief: ``prepare()`` polls until the chief has initialised the variables
(``SessionManager.wait_for_session``).
``should_stop()`` / ``request_stop()`` / ``stop()`` as in TF; ``stop()`` joins
the service threads and does NOT save a final checkpoint (TF semantics).
"""
from __future__ import annotations

import threading
import time

from .. import ckpt


class Supervisor:
    def __init__(self, is_chief: bool, logdir: str, *, state_fn, restore_fn, init_fn, wait_fn, var_list_fn, gs_fn,
                 save_model_secs: float = 60.0, save_summaries_secs: float = 120.0, max_to_keep: int = 5,
                 log=print):
        """
        state_fn()        -> (dict name -> CPU tensor in TF layout, global_step)
        gs_fn()           -> current global step (step-counter thread)
        restore_fn(d)     -> push a checkpoint dict to the model (chief)
        init_fn()         -> initialise the model's variables (chief, no checkpoint)
        wait_fn()         -> block until the chief initialised (non-chief)
        var_list_fn()     -> [(name, tf_dtype, shape)] for graph.pbtxt / events
        """
        self.is_chief = is_chief
        self.logdir = logdir
        self.state_fn, self.restore_fn, self.init_fn, self.wait_fn = state_fn, restore_fn, init_fn, wait_fn
        self.var_list_fn = var_list_fn
        self.gs_fn = gs_fn
        self.save_model_secs = save_model_secs
        self.save_summaries_secs = save_summaries_secs
        self.log = log
        self._stop = threading.Event()
        self._threads = []
        self.saver = ckpt.Saver(logdir, max_to_keep=max_to_keep) if is_chief else None
        self.events = None
        self.restored_from = None
        self.exception = None
        self._last_gs = None
        self.saves = 0
        self._ev_lock = threading.Lock()  # the step-counter thread and summary() share the writer

    # ---------------------------------------------------------------- setup
    def prepare(self):
        if not self.is_chief:
            self.wait_fn()
            return
        path = ckpt.latest_checkpoint(self.logdir)
        if path:
            self.restore_fn(ckpt.load_bundle(path))
            self.restored_from = path
        else:
            self.init_fn()
        vars_ = self.var_list_fn()
        ckpt.write_graph_pbtxt(self.logdir, vars_)
        self.events = ckpt.EventWriter(self.logdir)
        self.events.add_graph_of_variables(vars_)
        if self.save_model_secs and self.save_model_secs > 0:
            self._start(self._checkpoint_loop, "sv-checkpoint")
        if self.save_summaries_secs and self.save_summaries_secs > 0:
            self._start(self._step_counter_loop, "sv-step-counter")

    def _start(self, fn, name):
        t = threading.Thread(target=self._guard(fn), name=name, daemon=True)
        t.start()
        self._threads.append(t)

    def _guard(self, fn):
        def run():
            try:
                fn()
            except Exception as e:  # noqa: BLE001 - surfaced via should_stop()/stop()
                self.exception = e
                self.request_stop()
        return run

    # ---------------------------------------------------------------- loops
    def save_now(self):
        tensors, gs = self.state_fn()
        p = self.saver.save(tensors, gs)
        self.saves += 1
        return p

    def _checkpoint_loop(self):
        while not self._stop.is_set():
            self.save_now()
            if self._stop.wait(self.save_model_secs):
                return

    def _step_counter_loop(self):
        last_t, last_gs = time.time(), None
        while not self._stop.wait(self.save_summaries_secs):
            gs = self.gs_fn()
            now = time.time()
            if last_gs is not None and now > last_t:
                rate = (gs - last_gs) / (now - last_t)
                with self._ev_lock:
                    self.events.add_scalars(gs, {"global_step/sec": rate})
            last_t, last_gs = now, gs

    # ------------------------------------------------------------ control
    def should_stop(self) -> bool:
        return self._stop.is_set()

    def request_stop(self):
        self._stop.set()

    def summary(self, step, scalars: dict):
        """Append scalar summaries (losses, images/sec) to the chief's events file; a no-op on
        non-chief tasks (TF: only the chief's Supervisor owns a summary writer)."""
        if self.events is not None and scalars:
            with self._ev_lock:
                self.events.add_scalars(step, scalars)

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=60)
        self._threads.clear()
        if self.events is not None:
            with self._ev_lock:
                self.events.close()
            self.events = None
        if self.exception is not None:
            raise self.exception
