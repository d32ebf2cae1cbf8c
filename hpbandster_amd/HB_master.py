"""HpBandSter -- drop-in for hpbandster/HB_master.py.

Same constructor, budget ladder (HB_master.py:93-94), bracket sizes (HB_master.py:161-168), scheduling
loop, queue throttling and ``job_callback``.  The job transport is the reference's Pyro4 Dispatcher,
used untouched when ``hpbandster`` is installed; any object with its interface can be passed as
``dispatcher`` (e.g. ``hpbandster_amd.dispatch.SerialDispatcher``).  The compute this engine moves to
the MI355X lives in the config generator (KDE acquisition) and in ``SuccessiveHalving`` (promotion).
"""

import copy
import logging
import math
import os
import threading
import time

import numpy as np

from .HB_iteration import SuccessiveHalving
from .HB_result import HB_result


def hb_budgets(eta, min_budget, max_budget):
    """max_SH_iter and the geometric budget ladder (HB_master.py:93-94)."""
    max_SH_iter = -int(np.log(min_budget / max_budget) / np.log(eta)) + 1
    budgets = max_budget * np.power(eta, -np.linspace(max_SH_iter - 1, 0, max_SH_iter))
    return max_SH_iter, budgets


def hb_bracket(it, eta, max_SH_iter):
    """(s, ns) of Hyperband iteration ``it`` (HB_master.py:163-166)."""
    s = max_SH_iter - 1 - (it % max_SH_iter)
    n0 = int(np.floor((max_SH_iter) / (s + 1)) * eta ** s)
    ns = [max(int(n0 * (eta ** (-i))), 1) for i in range(s + 1)]
    return s, ns


class HpBandSter(object):
    def __init__(self, run_id, config_generator, working_directory='.', eta=3, min_budget=0.01, max_budget=1,
                 ping_interval=60, nameserver='127.0.0.1', ns_port=None, host=None, shutdown_workers=True,
                 job_queue_sizes=(0, np.inf), dynamic_queue_size=False, logger=None, dispatcher=None):
        self.working_directory = working_directory
        os.makedirs(self.working_directory, exist_ok=True)
        self.logger = logging.getLogger('hpbandster') if logger is None else logger
        self.config_generator = config_generator
        self.time_ref = None
        self.eta = eta
        self.min_budget = min_budget
        self.max_budget = max_budget
        self.max_SH_iter, self.budgets = hb_budgets(eta, min_budget, max_budget)
        self.iterations = []
        self.jobs = []
        self.num_running_jobs = 0
        self.job_queue_sizes = job_queue_sizes
        self.user_job_queue_sizes = job_queue_sizes
        self.dynamic_queue_size = dynamic_queue_size
        if job_queue_sizes[0] >= job_queue_sizes[1]:
            raise ValueError("The queue size range needs to be (min, max) with min<max!")
        self.thread_cond = threading.Condition()
        self.config = {'eta': eta, 'min_budget': min_budget, 'max_budget': max_budget, 'budgets': self.budgets,
                       'max_SH_iter': self.max_SH_iter, 'time_ref': self.time_ref}
        if dispatcher is None:
            try:
                from hpbandster.distributed.dispatcher import Dispatcher  # the reference's Pyro4 transport
            except ImportError as e:
                raise ImportError("no job dispatcher: install hpbandster (Pyro4 transport) or pass "
                                  "dispatcher=hpbandster_amd.dispatch.SerialDispatcher(compute)") from e
            dispatcher = Dispatcher
        if isinstance(dispatcher, type):
            self.dispatcher = dispatcher(self.job_callback, queue_callback=self.adjust_queue_size, run_id=run_id,
                                         ping_interval=ping_interval, nameserver=nameserver, ns_port=ns_port,
                                         host=host)
        else:
            self.dispatcher = dispatcher
            self.dispatcher.new_result_callback = self.job_callback
        self.dispatcher_thread = threading.Thread(target=self.dispatcher.run)
        self.dispatcher_thread.start()

    def shutdown(self, shutdown_workers=False):
        self.logger.debug('HBMASTER: shutdown initiated, shutdown_workers = %s' % (str(shutdown_workers)))
        self.dispatcher.shutdown(shutdown_workers)
        self.dispatcher_thread.join()

    def run(self, n_iterations, iteration_class=SuccessiveHalving, min_n_workers=1, iteration_class_kwargs={}):
        while self.dispatcher.number_of_workers() < min_n_workers:
            self.logger.debug('HBMASTER: only %i worker(s) available, waiting for at least %i.'
                              % (self.dispatcher.number_of_workers(), min_n_workers))
            time.sleep(1)
        if self.time_ref is None:
            self.time_ref = time.time()
            self.config['time_ref'] = self.time_ref
            self.logger.info('HBMASTER: starting run at %s' % (str(self.time_ref)))
        for it in range(len(self.iterations), len(self.iterations) + n_iterations):
            s, ns = hb_bracket(it, self.eta, self.max_SH_iter)
            self.iterations.append(iteration_class(iter_number=it, num_configs=ns, budgets=self.budgets[(-s - 1):],
                                                   config_sampler=self.config_generator.get_config,
                                                   **iteration_class_kwargs))
        while len(self.active_iterations()) > 0:
            for i in self.active_iterations():
                next_run = self.iterations[i].get_next_run()
                if next_run is not None:
                    self.logger.debug('HBMASTER: schedule new run for iteration %i' % i)
                    self._submit_job(*next_run)
                    break  # lower iterations first
        return HB_result([copy.deepcopy(i.data) for i in self.iterations], self.config)

    def adjust_queue_size(self, number_of_workers=None):
        if self.dynamic_queue_size:
            with self.thread_cond:
                nw = self.dispatcher.number_of_workers() if number_of_workers is None else number_of_workers
                self.job_queue_sizes = (self.user_job_queue_sizes[0] + nw, self.user_job_queue_sizes[1] + nw)
                self.logger.info('HBMASTER: adjusted queue size to %s' % str(self.job_queue_sizes))
                self.thread_cond.notify_all()

    def job_callback(self, job):
        self.logger.debug('job_callback for %s' % str(job.id))
        with self.thread_cond:
            self.num_running_jobs -= 1
            if self.num_running_jobs <= self.job_queue_sizes[0]:
                self.thread_cond.notify()
            self.iterations[job.id[0]].register_result(job)
        self.config_generator.new_result(job)

    def _submit_job(self, config_id, config, budget):
        with self.thread_cond:
            if self.num_running_jobs >= self.job_queue_sizes[1]:
                while self.num_running_jobs > self.job_queue_sizes[0]:
                    self.thread_cond.wait()
            self.num_running_jobs += 1
        self.dispatcher.submit_job(config_id, config=config, budget=budget, working_directory=self.working_directory)

    def active_iterations(self):
        return [idx for idx in range(len(self.iterations)) if not self.iterations[idx].is_finished]
