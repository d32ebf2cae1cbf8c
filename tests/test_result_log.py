"""Result log / HB_result against the reference's own files and API outputs.

tests/golden/e2e_log/{configs,results}.json were written by the reference's json_result_logger
(utils.py:7-75) during the reference's end-to-end toy run (gen_golden.py --only e2e), and
tests/golden/e2e_hb_result.json holds what the reference's logged_results_to_HB_result
(utils.py:78-126) and HB_result API (HB_result.py:80-272) returned on that log."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LOG = os.path.join(HERE, "e2e_log")


def _ref():
    with open(os.path.join(HERE, "e2e_hb_result.json")) as fh:
        return json.load(fh)


def _run_rec(r):
    return [list(r.config_id), r.budget, r.loss, r.info, r.time_stamps, r.error_logs]


def test_reload_and_api_match_reference():
    from hpbandster_amd.utils import logged_results_to_HB_result
    want = _ref()
    hr = logged_results_to_HB_result(LOG)
    assert json.loads(json.dumps(hr.HB_config)) == want["HB_config"]
    assert list(hr.get_incumbent_id()) == want["incumbent"]
    assert hr.num_iterations() == want["num_iterations"]
    for key, ab in (("trajectory_all", True), ("trajectory_max", False)):
        t = hr.get_incumbent_trajectory(all_budgets=ab)
        t["config_ids"] = [list(c) for c in t["config_ids"]]
        assert json.loads(json.dumps(t)) == want[key]
    assert json.loads(json.dumps([_run_rec(r) for r in hr.get_all_runs()])) == want["all_runs"]
    assert json.loads(json.dumps([_run_rec(r) for r in hr.get_all_runs(only_largest_budget=True)])) == \
        want["all_runs_largest"]
    lcs = [[list(k), v] for k, v in hr.get_learning_curves().items()]
    assert json.loads(json.dumps(lcs)) == want["learning_curves"]
    assert json.loads(json.dumps([[list(k), v] for k, v in hr.get_id2config_mapping().items()])) == want["id2config"]
    for k, runs in want["runs_by_id"].items():
        cid = tuple(json.loads(k))
        assert json.loads(json.dumps([_run_rec(r) for r in hr.get_runs_by_id(cid)])) == runs
    assert repr(hr.get_all_runs()[0]) == want["repr_first"]


class _Job(object):
    def __init__(self, id, config, budget, timestamps, result, exception):
        self.id, self.kwargs = id, {"config": config, "budget": budget}
        self.timestamps, self.result, self.exception = timestamps, result, exception


def test_logger_writes_the_reference_files(tmp_path):
    """Replaying the logged jobs (in the logged order) through this json_result_logger reproduces the
    reference's two files byte for byte."""
    from hpbandster_amd.utils import json_result_logger
    configs = {}
    with open(os.path.join(LOG, "configs.json")) as fh:
        for line in fh:
            cid, cfg = json.loads(line)
            configs[tuple(cid)] = cfg
    lg = json_result_logger(str(tmp_path))
    with open(os.path.join(LOG, "results.json")) as fh:
        for line in fh:
            cid, b, ts, res, exc = json.loads(line)
            lg(_Job(tuple(cid), configs[tuple(cid)], b, ts, res, exc))
    for fn in ("configs.json", "results.json"):
        assert open(os.path.join(str(tmp_path), fn)).read() == open(os.path.join(LOG, fn)).read(), fn


def test_trajectory_and_empty_runs_raise_like_reference():
    """HB_result on data without finished runs: get_incumbent_id is None, the trajectory raises
    IndexError as the reference's does (HB_result.py:150-155)."""
    import pytest
    from hpbandster_amd.HB_result import HB_result
    data = {(0, 0, 0): {"config": {}, "results": {1.0: None}, "time_stamps": {1.0: {"submitted": 1.0,
            "started": 2.0, "finished": 3.0}}, "exceptions": {1.0: "x"}}}
    hr = HB_result([data], {"max_budget": 1.0, "time_ref": 0.0})
    assert hr.get_incumbent_id() is None
    with pytest.raises(IndexError):
        hr.get_incumbent_trajectory()
    assert hr.get_learning_curves() == {(0, 0, 0): [[(1.0, None)]]}
