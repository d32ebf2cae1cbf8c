"""SuccessiveHalving / SuccessiveResampling -- drop-ins for hpbandster/HB_iteration.py.

Same state machine (QUEUED -> RUNNING -> REVIEW | CRASHED -> QUEUED/TERMINATED) and API
(``get_next_run``, ``register_result``, ``process_results``, ``add_configuration``); the ranking step
of ``process_results`` (``argsort(argsort(losses)) < k``, HB_iteration.py:179-182 and 239-242) runs
as the GPU segmented top-k of libhbx.so (``promote.advance_mask``).
"""

import numpy as np

from . import promote


class SuccessiveHalving(object):
    """One Hyperband bracket (reference HB_iteration.py:7-198)."""

    def __init__(self, iter_number, num_configs, budgets, config_sampler, device=None, batch_sampling=True):
        self.data = {}
        self.is_finished = False
        self.HB_iter = iter_number
        self.SH_iter = 0
        self.budgets = budgets
        self.num_configs = num_configs
        self.actual_num_configs = [0] * len(num_configs)
        self.config_sampler = config_sampler
        self.num_running = 0
        self.device = device
        # back-to-back requests are served from speculative batches when the sampler's
        # generator offers them (BOHB.get_config_batch_spec); each result is used only while it is exactly
        # the sequential call's (same model, same RNG states), else sampled afresh.  Batch sizes grow
        # geometrically (1, 2, 4, ...) while every result of the last batch was served and nothing changed
        # since; a batch cut short by a result (a model refit) or a draw in between falls back to single
        # calls -- so with one worker, where every request follows a refit, nothing is computed ahead -- and
        # each cut-short batch in a row doubles the run of undisturbed single calls the next batch waits for
        # (results arriving on the dispatcher thread between requests: batches of 2 cut short every other
        # call cost 12 % of a threaded HpBandSter.run, bench threaded_run)
        self.batch_sampling = batch_sampling
        self._spec = None
        self._fp = None   # after a single call: the generator's state fingerprint (BOHB.spec_fingerprint)
        self._next = 1    # size of the next speculative batch
        self._cut = 0     # speculative batches cut short in a row
        self._calm = 0    # single calls in a row with nothing changed between them
        gen = getattr(config_sampler, "__self__", None)  # resolved once: the sampler is fixed per instance
        ok = (batch_sampling and getattr(config_sampler, "__name__", "") == "get_config"
              and getattr(gen, "get_config_batch_spec", None) is not None)
        self._gen = gen if ok else None

    MAX_BATCH = 128

    def _sample(self, budget):
        gen = self._gen
        if gen is None or not gen.speculation_enabled():
            return self.config_sampler(budget)
        if self._spec is not None:
            r = self._spec.take()
            if r is not None:
                return r
            cont = self._spec.continues()
            self._next = min(2 * len(self._spec), self.MAX_BATCH) if cont else 1
            self._cut = 0 if cont else min(self._cut + 1, 6)
            self._calm = 0
            self._spec = None
        elif self._fp is not None:
            self._calm = self._calm + 1 if gen.spec_unchanged(self._fp) else 0
            self._next = 2 if self._calm >= (1 << self._cut) else 1
        self._fp = None
        remaining = self.num_configs[self.SH_iter] - self.actual_num_configs[self.SH_iter]
        size = min(remaining, self._next)
        if size > 1:
            spec = gen.get_config_batch_spec(budget, size)
            r = spec.take() if spec is not None else None
            if r is not None:
                self._spec = spec
                return r
            self._next = 1
        r = self.config_sampler(budget)
        self._fp = gen.spec_fingerprint()
        return r

    def add_configuration(self, config=None, config_info={}):
        if config is None:
            config, config_info = self._sample(self.budgets[self.SH_iter])
        if self.is_finished:
            raise RuntimeError("This HB iteration is finished, you can't  add more results!")
        if self.actual_num_configs[self.SH_iter] == self.num_configs[self.SH_iter]:
            raise RuntimeError("Can't add another configuration to SH_iteration %i in HB_iteration %i."
                               % (self.SH_iter, self.HB_iter))
        config_id = (self.HB_iter, self.SH_iter, self.actual_num_configs[self.SH_iter])
        self.data[config_id] = {
            'config': config, 'config_info': config_info, 'results': {}, 'time_stamps': {},
            'exceptions': {}, 'status': 'QUEUED', 'budget': self.budgets[self.SH_iter],
        }
        self.actual_num_configs[self.SH_iter] += 1
        return config_id

    def register_result(self, job):
        if self.is_finished:
            raise RuntimeError("This HB iteration is finished, you can't register more results!")
        config_id = job.id
        config = job.kwargs['config']
        budget = job.kwargs['budget']
        d = self.data[config_id]
        assert d['config'] == config, 'Configurations differ!'
        assert d['status'] == 'RUNNING', "Configuration wasn't scheduled for a run."
        assert d['budget'] == budget, 'Budgets differ (%f != %f)!' % (d['budget'], budget)
        d['time_stamps'][budget] = job.timestamps
        d['results'][budget] = job.result
        if (job.result is not None) and np.isfinite(job.result['loss']):
            d['status'] = 'REVIEW'
        else:
            d['status'] = 'CRASHED'
            d['exceptions'][budget] = {job.exception}
        self.num_running -= 1

    def get_next_run(self):
        if self.is_finished:
            return None
        for k, v in self.data.items():
            if v['status'] == 'QUEUED':
                assert v['budget'] == self.budgets[self.SH_iter], \
                    'Configuration budget does not align with current SH iteration!'
                v['status'] = 'RUNNING'
                self.num_running += 1
                return (k, v['config'], v['budget'])
        if self.actual_num_configs[self.SH_iter] < self.num_configs[self.SH_iter]:
            self.add_configuration()
            return self.get_next_run()
        if self.num_running == 0:
            self.process_results()
            return self.get_next_run()
        return None

    def _advance_threshold(self):
        """k of the top-k: configurations ranked below it advance."""
        return self.num_configs[self.SH_iter]

    def process_results(self):
        """HB_iteration.py:149-190: rank the REVIEW configurations of this stage on the GPU
        (promote.advance_mask), mark the top k QUEUED at the next budget, the rest TERMINATED.  One
        pass over the dict for the ids and budgets, one for the losses, one for the updates."""
        self.SH_iter += 1
        config_ids, budgets = [], []
        for cid, d in self.data.items():
            if d['status'] == 'REVIEW':
                config_ids.append(cid)
                budgets.append(d['budget'])
        if self.SH_iter >= len(self.num_configs):
            self.cleanup()
            return
        if len(config_ids) > 0:
            if len(set(budgets)) > 1:
                raise RuntimeError('Not all configurations have the same budget!')
            budget = budgets[0]
            data = self.data
            losses = np.fromiter((data[cid]['results'][budget]['loss'] for cid in config_ids), dtype=np.float64,
                                 count=len(config_ids))
            advance = promote.advance_mask(losses, self._advance_threshold(), device=self.device)
            nb = self.budgets[self.SH_iter]
            moved = 0
            for cid, a in zip(config_ids, advance.tolist()):
                d = data[cid]
                if a:
                    d['status'] = 'QUEUED'
                    d['budget'] = nb
                    moved += 1
                else:
                    d['status'] = 'TERMINATED'
            self.actual_num_configs[self.SH_iter] += moved

    def cleanup(self):
        self.is_finished = True
        for k, v in self.data.items():
            assert v['status'] in ['TERMINATED', 'REVIEW', 'CRASHED'], 'Configuration has not finshed yet!'
            del v['status']
            del v['budget']


class SuccessiveResampling(SuccessiveHalving):
    """Advance the best half of the next stage's size, refill the rest with new samples
    (reference HB_iteration.py:203-250)."""
    resampling_rate = 0.5
    min_samples_advance = 1

    def _advance_threshold(self):
        return max(self.min_samples_advance, self.num_configs[self.SH_iter] * (1 - self.resampling_rate))
