"""Result logging, format-compatible with the reference (hpbandster/utils.py:7-126).

``configs.json`` holds one JSON line ``[config_id, config]`` per configuration, ``results.json`` one
line ``[config_id, budget, timestamps, result, exception]`` per finished run -- the on-disk format
of the reference, so logs written by either implementation load with either loader.
"""

import json
import os


class json_result_logger(object):
    def __init__(self, directory, overwrite=False):
        os.makedirs(directory, exist_ok=True)
        self.config_fn = os.path.join(directory, 'configs.json')
        self.results_fn = os.path.join(directory, 'results.json')
        for fn in (self.config_fn, self.results_fn):
            try:
                with open(fn, 'x'):
                    pass
            except FileExistsError:
                if overwrite:
                    with open(fn, 'w'):
                        pass
                else:
                    raise FileExistsError('The file %s already exists.' % fn)
        self.config_ids = set()

    def __call__(self, job):
        if job.id not in self.config_ids:
            self.config_ids.add(job.id)
            with open(self.config_fn, 'a') as fh:
                fh.write(json.dumps([job.id, job.kwargs['config']]))
                fh.write('\n')
        with open(self.results_fn, 'a') as fh:
            fh.write(json.dumps([job.id, job.kwargs['budget'], job.timestamps, job.result, job.exception]))
            fh.write("\n")


def logged_results_to_HB_result(directory):
    """Reload a json_result_logger directory into an HB_result (reference utils.py:78-126)."""
    from .HB_result import HB_result
    data = {}
    time_ref = float('inf')
    budget_set = set()
    with open(os.path.join(directory, 'configs.json')) as fh:
        for line in fh:
            config_id, config = json.loads(line)
            data[tuple(config_id)] = {'config': config, 'results': {}, 'time_stamps': {}, 'exceptions': {}}
    with open(os.path.join(directory, 'results.json')) as fh:
        for line in fh:
            config_id, budget, time_stamps, result, exception = json.loads(line)
            cid = tuple(config_id)
            data[cid]['time_stamps'][budget] = time_stamps
            data[cid]['results'][budget] = result
            data[cid]['exceptions'][budget] = exception
            budget_set.add(budget)
            time_ref = min(time_ref, time_stamps['submitted'])
    budget_list = sorted(budget_set)
    HB_config = {
        'eta': None if len(budget_list) < 2 else budget_list[1] / budget_list[0],
        'min_budget': min(budget_set), 'max_budget': max(budget_set), 'budgets': budget_list,
        'max_SH_iter': len(budget_set), 'time_ref': time_ref,
    }
    return HB_result([data], HB_config)
