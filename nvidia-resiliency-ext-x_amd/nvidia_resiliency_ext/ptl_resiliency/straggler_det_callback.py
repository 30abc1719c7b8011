"""PTL ``StragglerDetectionCallback`` on the HIP-backed Detector
(reference: ptl_resiliency/straggler_det_callback.py:36-258).

Same constructor arguments, hooks and side effects as the reference:

* ``setup``: ``Detector.initialize(scores, gather_on_rank0=True, profiling_interval,
  report_time_interval)`` and wrap ``trainer.strategy.training_step`` in a detection
  section (straggler_det_callback.py:97-106);
* ``on_train_batch_end``: ``generate_report_if_interval_elapsed``; rank 0 identifies the
  stragglers, logs them (WARNING), prints the best/worst scores (INFO), logs min/median/max
  to the PTL loggers; when the interval elapsed and ``stop_if_detected``, rank 0's verdict
  is broadcast and a positive one stops the trainer (:213-258);
* ``teardown``: ``Detector.shutdown``.

The reference raises ImportError without Lightning.  Lightning is not part of this image,
so the base class falls back to a plain object with the same hook names: any training loop
(or a test) can call the hooks directly.  With ``lightning`` or ``pytorch_lightning``
installed the callback is a real ``Callback`` subclass.
"""
from __future__ import annotations

import importlib.util
import logging
import sys
import time
from typing import Dict, List, Mapping, Optional

import torch

import nvidia_resiliency_ext.straggler as straggler
from nvidia_resiliency_ext.common.device_utils import get_current_device


def _lightning_callback_base():
    for mod in ("lightning.pytorch.callbacks", "pytorch_lightning.callbacks"):
        top = mod.split(".")[0]
        if importlib.util.find_spec(top) is not None:
            return importlib.import_module(mod).Callback
    return None


_Base = _lightning_callback_base()
LIGHTNING_AVAILABLE = _Base is not None
if _Base is None:
    class _Base:  # type: ignore[no-redef]
        """Hook-compatible stand-in for ``lightning.pytorch.callbacks.Callback``."""

        def setup(self, trainer, pl_module, stage):
            pass

        def teardown(self, trainer, pl_module, stage):
            pass

        def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx):
            pass


_REL = "relative_perf_scores"
_IND = "individual_perf_scores"


class StragglerDetectionCallback(_Base):
    def __init__(self, report_time_interval: float, calc_relative_gpu_perf: bool,
                 calc_individual_gpu_perf: bool, num_gpu_perf_scores_to_print: int,
                 gpu_relative_perf_threshold: float, gpu_individual_perf_threshold: float,
                 stop_if_detected: bool, enable_ptl_logging: bool, profiling_interval: int = 1,
                 logger_name: Optional[str] = "nemo_logger.StragglerDetectionCallback"):
        """See the reference docstring (straggler_det_callback.py:49-75).  Raises ValueError
        when neither relative nor individual scores are requested."""
        self.initialized = False
        self.logger = logging.getLogger(logger_name)
        self.report_time_interval = report_time_interval
        self.calc_relative_gpu_perf = calc_relative_gpu_perf
        self.calc_individual_gpu_perf = calc_individual_gpu_perf
        self.num_gpu_perf_scores_to_print = num_gpu_perf_scores_to_print
        self.gpu_relative_perf_threshold = gpu_relative_perf_threshold
        self.gpu_individual_perf_threshold = gpu_individual_perf_threshold
        self.stop_if_detected = stop_if_detected
        self.enable_ptl_logging = enable_ptl_logging
        self.profiling_interval = profiling_interval
        self.scores_to_compute: List[str] = (
            ([_REL] if calc_relative_gpu_perf else []) + ([_IND] if calc_individual_gpu_perf else []))
        if not self.scores_to_compute:
            raise ValueError("No straggler performance scores specified. Check if "
                             "calc_relative_gpu_perf=True or calc_individual_gpu_perf=True")
        self.interval_est_was_reset = False

    # -- lifecycle -------------------------------------------------------------------------
    def _wrap_ptl_callables(self, trainer):
        assert getattr(trainer.strategy, "training_step", None), \
            f"{type(trainer.strategy)} does not have 'training_step' method."
        straggler.Detector.wrap_callables(
            callable_ids=[straggler.CallableId(trainer.strategy, "training_step")])

    def setup(self, trainer, pl_module, stage):
        if self.initialized:
            return
        straggler.Detector.initialize(scores_to_compute=self.scores_to_compute,
                                      gather_on_rank0=True,
                                      profiling_interval=self.profiling_interval,
                                      report_time_interval=self.report_time_interval)
        self._wrap_ptl_callables(trainer)
        self.initialized = True

    def teardown(self, trainer, pl_module, stage):
        if self.initialized:
            straggler.Detector.shutdown()
            self.initialized = False

    # -- report handling -------------------------------------------------------------------
    def _print_stragglers(self, stragglers):
        rel = stragglers["straggler_gpus_relative"]
        ind = stragglers["straggler_gpus_individual"]
        if rel:
            self.logger.warning("STRAGGLER DETECTION WARNING: Some GPUs have worse relative "
                                f"performance. Affected ranks: {rel}")
        if ind:
            self.logger.warning("STRAGGLER DETECTION WARNING: Some GPUs performance dropped. "
                                f"Affected ranks: {ind}")

    @staticmethod
    def _format_gpu_scores(rank_to_score: Mapping[int, float], rank_to_node: Mapping[int, str],
                           num_best: int = 3, num_worst: int = 3) -> str:
        """Worst ``num_worst`` (ascending score) then best ``num_best`` (descending); every
        rank, ascending, when there are at most num_best + num_worst (:127-145).  Ties order
        by rank as the reference's ``sort(reverse=True)`` over (score, rank) pairs does."""
        ranked = sorted(((s, r) for r, s in rank_to_score.items()), reverse=True)

        def line(s, r):
            return f"  Rank={r} Node={rank_to_node[r]} Score={s:.2f}\n"

        n = len(ranked)
        if n <= num_best + num_worst:
            return "".join(line(s, r) for s, r in reversed(ranked))
        worst = ranked[-num_worst:]  # num_worst == 0 selects every rank, as in the reference
        out = [f" Worst performing {num_worst}/{n} ranks:\n"]
        out += [line(s, r) for s, r in reversed(worst)]
        out.append(f" Best performing {num_best}/{n} ranks:\n")
        out += [line(s, r) for s, r in ranked[:num_best]]
        return "".join(out)

    def _score_views(self, report):
        views = []
        if self.calc_relative_gpu_perf:
            views.append(("relative", "gpu_relative_perf", report.gpu_relative_perf_scores))
        if self.calc_individual_gpu_perf:
            views.append(("individual", "gpu_individual_perf", report.gpu_individual_perf_scores))
        return views

    def _print_gpu_scores(self, report):
        assert self.num_gpu_perf_scores_to_print > 0
        k = self.num_gpu_perf_scores_to_print
        for kind, _, scores in self._score_views(report):
            text = self._format_gpu_scores(scores, report.rank_to_node, num_best=k, num_worst=k)
            self.logger.info(f"\nGPU {kind} performance:\n{text}")

    def _log_gpu_perf_scores(self, pl_module, rank_to_score, rank_to_node, score_prefix):
        """min / median (lower, torch.median) / max of the scores as float32, NaN when empty,
        through ``pl_module.log_dict`` (:166-186); logging errors are reported, not raised."""
        lo = med = hi = float("nan")
        vals = list(rank_to_score.values())
        if vals:
            t = torch.tensor(vals, dtype=torch.float32)
            lo, med, hi = torch.min(t).item(), torch.median(t).item(), torch.max(t).item()
        scores_log: Dict[str, float] = {f"{score_prefix}/min": lo, f"{score_prefix}/median": med,
                                        f"{score_prefix}/max": hi}
        try:
            pl_module.log_dict(scores_log, logger=True, batch_size=1, rank_zero_only=True)
        except Exception as e:  # noqa: BLE001 - the reference logs and continues
            self.logger.error(f"Failed to log GPU performance scores: {e}")

    def _log_gpu_scores(self, pl_module, report):
        assert self.enable_ptl_logging is True
        for _, prefix, scores in self._score_views(report):
            self._log_gpu_perf_scores(pl_module, rank_to_score=scores,
                                      rank_to_node=report.rank_to_node, score_prefix=prefix)

    def _handle_straggler_report(self, pl_module, report) -> bool:
        stragglers = report.identify_stragglers(
            gpu_rel_threshold=self.gpu_relative_perf_threshold,
            gpu_indiv_threshold=self.gpu_individual_perf_threshold)
        found = bool(stragglers["straggler_gpus_relative"]
                     or stragglers["straggler_gpus_individual"])
        if found:
            self._print_stragglers(stragglers)
        if self.num_gpu_perf_scores_to_print > 0:
            self._print_gpu_scores(report)
        if self.enable_ptl_logging:
            self._log_gpu_scores(pl_module, report)
        return found

    def _gather_flag_from_rank0(self, flag: bool) -> bool:
        t = torch.tensor([1.0 if flag else 0.0], device=get_current_device(), dtype=torch.float32)
        torch.distributed.broadcast(t, 0)
        return bool(t.item() > 0)

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx):
        t0 = time.monotonic()
        report = straggler.Detector.generate_report_if_interval_elapsed()
        found = False
        if trainer.global_rank == 0 and report:
            # gather_on_rank0=True: only rank 0 holds the report
            found = self._handle_straggler_report(pl_module, report)
        if straggler.Detector.is_interval_elapsed():
            if self.stop_if_detected and self._gather_flag_from_rank0(found):
                self._stop_training(trainer)
            self.logger.info(f"Straggler report processing time: {time.monotonic() - t0:.3f} sec.")

    def _stop_training(self, trainer) -> None:
        """Stop the trainer; with a checkpoint callback, save the last checkpoint (waiting for
        an async save) and exit(1) (:244-258)."""
        self.logger.error("Detected stragglers. Terminating training...")
        trainer.should_stop = True
        ckpt = trainer.checkpoint_callback
        if not ckpt:
            return
        ckpt._save_last_checkpoint(trainer, ckpt._monitor_candidates(trainer))
        cio = trainer.strategy.checkpoint_io
        if hasattr(cio, "maybe_finalize_save_checkpoint"):
            self.logger.info("Async checkpointing detected, waiting for it to complete...")
            cio.maybe_finalize_save_checkpoint(blocking=True)
        sys.exit(1)
