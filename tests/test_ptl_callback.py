"""StragglerDetectionCallback (ptl_resiliency/straggler_det_callback.py) -- the reference's
tests/ptl_resiliency/unit/test_straggler_det_callback.py restated without Lightning (absent
from this image): a minimal training loop drives the same hooks a ``pl.Trainer`` calls
(setup -> strategy.training_step + on_train_batch_end per batch -> teardown).

CPU: constructor errors, score formatting, report handling and PTL logging, the stop flag
broadcast from rank 0 (gloo, ws=2) with the Detector calls replaced by fakes.
GPU: the reference's two fitting tests (scores printed / logged) on the HIP Detector.
"""
import json
import logging
import math
import os
import subprocess
import sys
import time

import pytest

from _mp import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cb(**kw):
    from nvidia_resiliency_ext.ptl_resiliency import StragglerDetectionCallback

    args = dict(report_time_interval=1.0, calc_relative_gpu_perf=True,
                calc_individual_gpu_perf=True, num_gpu_perf_scores_to_print=1,
                gpu_relative_perf_threshold=0.0, gpu_individual_perf_threshold=0.0,
                enable_ptl_logging=False, stop_if_detected=False, logger_name="test_logger")
    args.update(kw)
    return StragglerDetectionCallback(**args)


class _ListHandler(logging.Handler):
    def __init__(self):
        super().__init__(logging.DEBUG)
        self.records = []

    def emit(self, record):
        self.records.append((record.levelname, record.getMessage()))

    def text(self):
        return "\n".join(m for _, m in self.records)


@pytest.fixture
def log_capture():
    lg = logging.getLogger("test_logger")
    h = _ListHandler()
    lg.addHandler(h)
    old = lg.level
    lg.setLevel(logging.DEBUG)
    yield h
    lg.removeHandler(h)
    lg.setLevel(old)


class _Module:
    """Stands in for a LightningModule: log_dict collects what PTL loggers would get."""

    def __init__(self, fail=False):
        self.logged = []
        self.fail = fail

    def log_dict(self, d, logger=True, batch_size=1, rank_zero_only=True):
        if self.fail:
            raise RuntimeError("no logger attached")
        assert logger and batch_size == 1 and rank_zero_only
        self.logged.append(dict(d))


def _report(rel, ind, nodes=None):
    from nvidia_resiliency_ext.straggler import Report

    nodes = nodes or {r: f"node{r // 2}" for r in set(rel) | set(ind)}
    return Report(gpu_relative_perf_scores=rel, section_relative_perf_scores={},
                  gpu_individual_perf_scores=ind, section_individual_perf_scores={},
                  rank_to_node=nodes, local_section_summaries={}, local_kernel_summaries={},
                  generate_report_elapsed_time=0.0, gather_on_rank0=True, rank=0)


# ------------------------------------------------------------------------------------- CPU
def test_requires_some_scores():
    with pytest.raises(ValueError):
        _cb(calc_relative_gpu_perf=False, calc_individual_gpu_perf=False)
    assert _cb(calc_individual_gpu_perf=False).scores_to_compute == ["relative_perf_scores"]
    assert _cb().scores_to_compute == ["relative_perf_scores", "individual_perf_scores"]


def test_format_gpu_scores_all_and_best_worst():
    from nvidia_resiliency_ext.ptl_resiliency import StragglerDetectionCallback as C

    nodes = {r: f"n{r}" for r in range(8)}
    few = C._format_gpu_scores({0: 0.5, 1: 1.0, 2: 0.75}, nodes, num_best=2, num_worst=2)
    assert few == ("  Rank=0 Node=n0 Score=0.50\n  Rank=2 Node=n2 Score=0.75\n"
                   "  Rank=1 Node=n1 Score=1.00\n")
    scores = {0: 0.9, 1: 0.2, 2: 1.0, 3: 0.4, 4: 0.95, 5: 0.6, 6: 0.3}
    txt = C._format_gpu_scores(scores, nodes, num_best=2, num_worst=3)
    assert txt == (" Worst performing 3/7 ranks:\n"
                   "  Rank=1 Node=n1 Score=0.20\n  Rank=6 Node=n6 Score=0.30\n"
                   "  Rank=3 Node=n3 Score=0.40\n"
                   " Best performing 2/7 ranks:\n"
                   "  Rank=2 Node=n2 Score=1.00\n  Rank=4 Node=n4 Score=0.95\n")
    # ties: (score, rank) pairs sorted descending -> the higher rank is "better"
    tie = C._format_gpu_scores({0: 0.5, 1: 0.5, 2: 0.5}, nodes, num_best=1, num_worst=1)
    assert tie.splitlines()[1] == "  Rank=0 Node=n0 Score=0.50"
    assert tie.splitlines()[3] == "  Rank=2 Node=n2 Score=0.50"


def test_handle_report_prints_and_warns(log_capture):
    cb = _cb(gpu_relative_perf_threshold=0.7, gpu_individual_perf_threshold=0.7)
    mod = _Module()
    found = cb._handle_straggler_report(mod, _report({0: 1.0, 1: 0.5}, {0: 0.9, 1: 1.0}))
    assert found
    warns = [m for lv, m in log_capture.records if lv == "WARNING"]
    assert len(warns) == 1 and "worse relative performance" in warns[0] and "rank=1" in warns[0]
    assert "GPU relative performance" in log_capture.text()
    assert "GPU individual performance" in log_capture.text()
    assert mod.logged == []  # enable_ptl_logging=False


def test_handle_report_quiet_without_stragglers(log_capture):
    cb = _cb(num_gpu_perf_scores_to_print=0, enable_ptl_logging=True,
             calc_individual_gpu_perf=False)
    mod = _Module()
    assert not cb._handle_straggler_report(mod, _report({0: 1.0, 1: 0.9}, {}))
    assert log_capture.records == []
    assert mod.logged == [{"gpu_relative_perf/min": pytest.approx(0.9),
                           "gpu_relative_perf/median": pytest.approx(0.9),
                           "gpu_relative_perf/max": 1.0}]


def test_ptl_logging_median_is_lower_and_errors_are_logged(log_capture):
    cb = _cb(enable_ptl_logging=True, num_gpu_perf_scores_to_print=0)
    mod = _Module()
    cb._log_gpu_scores(mod, _report({0: 0.25, 1: 1.0, 2: 0.5, 3: 0.75}, {}))
    rel, ind = mod.logged
    assert rel == {"gpu_relative_perf/min": 0.25, "gpu_relative_perf/median": 0.5,
                   "gpu_relative_perf/max": 1.0}
    assert all(math.isnan(v) for v in ind.values()) and len(ind) == 3
    cb._log_gpu_scores(_Module(fail=True), _report({0: 1.0}, {0: 1.0}))
    assert [lv for lv, _ in log_capture.records] == ["ERROR", "ERROR"]


def test_stop_flag_is_broadcast_from_rank0():
    res = run_world(2, "_callback_workers", "stop_flag_world")
    assert res[0] == {"should_stop": True, "reports": 1} and res[1]["should_stop"] is True


def test_no_stop_without_stragglers_or_when_disabled():
    res = run_world(2, "_callback_workers", "stop_flag_world", rel_score=0.99)
    assert res[0]["should_stop"] is False and res[1]["should_stop"] is False
    res = run_world(2, "_callback_workers", "stop_flag_world", stop_if_detected=False)
    assert res[0]["should_stop"] is False and res[1]["should_stop"] is False


# ------------------------------------------------------------------------------------- GPU
class _Strategy:
    def __init__(self, model, opt):
        self.model, self.opt = model, opt

    def training_step(self, batch, batch_idx):
        import torch

        x, y = batch
        loss = torch.nn.functional.cross_entropy(self.model(x), y)
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss


class _Trainer:
    global_rank = 0
    should_stop = False
    checkpoint_callback = None

    def __init__(self, strategy):
        self.strategy = strategy


def _fit(cb, seconds):
    """The Trainer.fit hook sequence, batch size 4 of ones (as the reference's OnesDataset)."""
    import torch

    torch.manual_seed(1234)
    dev = torch.device("cuda:0")
    model = torch.nn.Sequential(torch.nn.Linear(32, 16), torch.nn.ReLU(),
                                torch.nn.Linear(16, 10)).to(dev)
    trainer = _Trainer(_Strategy(model, torch.optim.Adam(model.parameters(), lr=1e-3)))
    module = _Module()
    x = torch.ones(4, 32, device=dev)
    y = torch.ones(4, 10, device=dev)
    cb.setup(trainer, module, "fit")
    try:
        t_end = time.monotonic() + seconds
        i = 0
        while time.monotonic() < t_end and not trainer.should_stop:
            out = trainer.strategy.training_step((x, y), i)
            cb.on_train_batch_end(trainer, module, out, (x, y), i)
            i += 1
    finally:
        cb.teardown(trainer, module, "fit")
    return module, i


def _fit_in_child(kind):
    """Run one fitting scenario in a fresh interpreter: kernel-dispatch capture is configured
    before the process's first HIP call (cupti.enable_capture), as a training script does
    by initialising the Detector before touching the GPU -- this pytest process has long
    initialised the runtime, so a Detector created here would capture nothing."""
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"), os.path.join(ROOT, "tests"),
         os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), kind], capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _child_main(kind):
    from nvidia_resiliency_ext.straggler import cupti

    assert cupti.enable_capture(), "capture must configure in a fresh process"
    from nvidia_resiliency_ext import straggler

    lg = logging.getLogger("test_logger")
    h = _ListHandler()
    lg.addHandler(h)
    lg.setLevel(logging.DEBUG)
    if kind == "print":
        module, iters = _fit(_cb(num_gpu_perf_scores_to_print=1, enable_ptl_logging=False), 3.0)
    else:
        module, iters = _fit(_cb(num_gpu_perf_scores_to_print=0, enable_ptl_logging=True), 3.0)
    print(json.dumps({"iters": iters, "log": h.text(), "logged": module.logged,
                      "initialized": bool(straggler.Detector.initialized),
                      "capture": bool(cupti.capture_available())}))


@pytest.mark.gpu
def test_prints_perf_scores_when_fitting():
    res = _fit_in_child("print")
    assert res["capture"] and res["iters"] > 16
    txt = res["log"]
    assert "GPU relative" in txt and "GPU individual" in txt
    assert "Straggler report processing time" in txt
    assert "Score=1.00" in txt  # one rank: relative score against itself
    assert res["logged"] == []
    assert not res["initialized"]


@pytest.mark.gpu
def test_logs_perf_scores_when_fitting():
    res = _fit_in_child("log")
    assert res["capture"]
    txt = res["log"]
    assert "GPU relative" not in txt and "GPU individual" not in txt
    logged = res["logged"]
    assert logged, "no scores reached the PTL loggers"
    keys = set().union(*logged)
    assert {"gpu_relative_perf/median", "gpu_individual_perf/max"} <= keys
    # one rank: relative scores are 1.0 (against itself); individual scores are 1.0 on
    # first sight and hist/MED <= 1 afterwards (reporting.py:298-314: history = running min)
    for d in logged:
        for k, v in d.items():
            if k.startswith("gpu_relative_perf/"):
                assert v == 1.0, (k, v, logged)
            else:
                assert 0.0 < v <= 1.0, (k, v, logged)
    assert logged[1]["gpu_individual_perf/max"] == 1.0  # the first report


@pytest.mark.gpu
def test_training_step_is_wrapped_in_a_detection_section():
    from nvidia_resiliency_ext import straggler

    cb = _cb(report_time_interval=1e9)
    import torch

    model = torch.nn.Linear(32, 10).cuda()
    strategy = _Strategy(model, torch.optim.SGD(model.parameters(), lr=0.1))
    trainer = _Trainer(strategy)
    original = strategy.training_step
    cb.setup(trainer, _Module(), "fit")
    try:
        assert strategy.training_step is not original
        batch = (torch.ones(4, 32, device="cuda"), torch.ones(4, 10, device="cuda"))
        for i in range(3):
            strategy.training_step(batch, i)
        sec = straggler.Detector.custom_sections["_Strategy.training_step"]
        assert sec.total_entry_cnt == 3 and len(sec.cpu_elapsed_times) == 3
    finally:
        cb.teardown(trainer, _Module(), "fit")
    assert strategy.training_step == original


if __name__ == "__main__":
    _child_main(sys.argv[1])
