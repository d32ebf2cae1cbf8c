"""HB_result -- the object HpBandSter.run returns (same API as hpbandster/HB_result.py:64-272).

Post-hoc analysis only (no GPU work): incumbent, incumbent trajectory, runs per configuration,
learning curves, id->config mapping.  Time stamps are made relative to ``HB_config['time_ref']``.
"""

import copy


class Run(object):
    """One evaluation of one configuration on one budget."""

    def __init__(self, config_id, budget, loss, info, time_stamps, error_logs):
        self.config_id = config_id
        self.budget = budget
        self.error_logs = error_logs
        self.loss = loss
        self.info = info
        self.time_stamps = time_stamps

    def __repr__(self):  # the reference's format (HB_result.py:17-24)
        return ("config_id: %s\t" % (self.config_id,) + "budget: %f\t" % self.budget + "loss: %s\n" % self.loss +
                "time_stamps: {submitted} (submitted), {started} (started), {finished} (finished)\n".format(
                    **self.time_stamps) + "info: %s\n" % self.info)

    def __getitem__(self, k):  # dictionary-style access, as the reference allows
        return getattr(self, k)


run = Run  # reference name


def extract_HB_learning_curves(runs):
    """Learning curve = (budget, loss) of every run by budget, crashed ones (loss None) included
    (HB_result.py:33-58)."""
    sr = sorted(runs, key=lambda r: r.budget)
    return [[(r.budget, r.loss) for r in sr]]


class HB_result(object):
    def __init__(self, HB_iteration_data, HB_config):
        self.data = HB_iteration_data
        self.HB_config = HB_config
        self._merge_results()

    def __getitem__(self, k):
        return self.data[k]

    def get_incumbent_id(self):
        """Config id with the smallest loss among runs on the maximum budget (None if none)."""
        best = []
        for k, v in self.data.items():
            res = v['results'].get(self.HB_config['max_budget'])
            if res is not None:
                best.append((res['loss'], k))
        return min(best)[1] if best else None

    def get_runs_by_id(self, config_id):
        d = self.data[config_id]
        runs = []
        for b in d['results'].keys():
            try:
                err = d['exceptions'].get(b, None)
                r = d['results'][b]
                if r is None:
                    runs.append(Run(config_id, b, None, None, d['time_stamps'][b], err))
                else:
                    runs.append(Run(config_id, b, r['loss'], r['info'], d['time_stamps'][b], err))
            except Exception:  # the reference skips any malformed entry (HB_result.py:180-181)
                pass
        runs.sort(key=lambda r: r.budget)
        return runs

    def get_all_runs(self, only_largest_budget=False):
        out = []
        for k in self.data.keys():
            runs = self.get_runs_by_id(k)
            if runs:
                out.extend(runs[-1:] if only_largest_budget else runs)
        return out

    def get_incumbent_trajectory(self, all_budgets=True):
        all_runs = self.get_all_runs(not all_budgets)
        if not all_budgets:
            all_runs = [r for r in all_runs if r.budget == self.HB_config['max_budget']]
        all_runs.sort(key=lambda r: r.time_stamps['finished'])
        out = {'config_ids': [], 'times_finished': [], 'budgets': [], 'losses': []}
        current = float('inf')
        for r in all_runs:
            if r.loss is None:
                continue
            if r.loss < current:
                current = r.loss
                out['config_ids'].append(r.config_id)
                out['times_finished'].append(r.time_stamps['finished'])
                out['budgets'].append(r.budget)
                out['losses'].append(r.loss)
        # the final point repeats the incumbent at the last finish time; like the reference this raises
        # IndexError when no run finished (HB_result.py:150-155)
        out['config_ids'].append(out['config_ids'][-1])
        out['times_finished'].append(all_runs[-1].time_stamps['finished'])
        out['budgets'].append(out['budgets'][-1])
        out['losses'].append(out['losses'][-1])
        return out

    def get_learning_curves(self, lc_extractor=extract_HB_learning_curves, config_ids=None):
        config_ids = self.data.keys() if config_ids is None else config_ids
        return {cid: lc_extractor(self.get_runs_by_id(cid)) for cid in config_ids}

    def get_id2config_mapping(self):
        out = {}
        for k, v in self.data.items():
            out[k] = {'config': copy.deepcopy(v['config'])}
            if 'config_info' in v:
                out[k]['config_info'] = copy.deepcopy(v['config_info'])
        return out

    def _merge_results(self):
        merged = {}
        for it in self.data:
            merged.update(it)
        for k, v in merged.items():
            for b, ts in v['time_stamps'].items():
                for kk, t in ts.items():
                    merged[k]['time_stamps'][b][kk] = t - self.HB_config['time_ref']
        self.data = merged

    def num_iterations(self):
        return max(k[0] for k in self.data.keys()) + 1
