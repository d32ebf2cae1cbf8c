"""Job record and an in-process serial dispatcher.

``Job`` has the fields of the reference's dispatcher Job (hpbandster/distributed/dispatcher.py:9-32).
The Pyro4 dispatcher/worker layer of the reference is coordination, not compute, and stays as it
is; ``HpBandSter`` uses it unchanged when hpbandster is installed.  ``SerialDispatcher`` runs jobs
synchronously in the calling thread (tests, examples, single-process use).
"""

import time


class Job(object):
    def __init__(self, id, *args, **kwargs):
        self.id = id
        self.args = args
        self.kwargs = kwargs
        self.timestamps = {}
        self.result = None
        self.exception = None
        self.worker_name = None

    def time_it(self, which_time):
        self.timestamps[which_time] = time.time()

    def __repr__(self):
        return ("job_id: " + str(self.id) + "\n" + "args: " + str(self.args) + "\n" + "kwargs: " +
                str(self.kwargs) + "\n" + "result: " + str(self.result) + "\n" + "exception: " +
                str(self.exception) + "\n")


class SerialDispatcher(object):
    """Dispatcher-compatible object that evaluates ``compute(config, budget, working_directory)``
    immediately and reports the result through the master's callback."""

    def __init__(self, compute, new_result_callback=None, queue_callback=None, **kwargs):
        self.compute = compute
        self.new_result_callback = new_result_callback

    def run(self):
        return

    def number_of_workers(self):
        return 1

    def shutdown(self, shutdown_workers=False):
        return

    def submit_job(self, id, **kwargs):
        job = Job(id, **kwargs)
        job.time_it('submitted')
        job.time_it('started')
        try:
            job.result = self.compute(config=kwargs['config'], budget=kwargs['budget'],
                                      working_directory=kwargs.get('working_directory', '.'))
        except Exception as e:  # a failing evaluation is a CRASHED run, like a worker exception
            job.exception = repr(e)
            job.result = None
        job.time_it('finished')
        if self.new_result_callback is not None:
            self.new_result_callback(job)
        return job


class ThreadedDispatcher(object):
    """Dispatcher-compatible object with ``n_workers`` in-process worker threads: ``submit_job`` queues the job,
    a worker thread evaluates ``compute``, and the dispatcher's own thread (``run``, started by HpBandSter)
    reports each finished job through the master's callback -- results arrive on the dispatcher thread while
    the master loop requests runs, as with the reference's Pyro4 dispatcher (hpbandster/distributed/
    dispatcher.py: job_callback runs in the dispatcher's thread)."""

    def __init__(self, compute, n_workers=8, new_result_callback=None, queue_callback=None, **kwargs):
        import queue
        import threading
        self.compute = compute
        self.n_workers = int(n_workers)
        self.new_result_callback = new_result_callback
        self.queue_callback = queue_callback
        self._jobs = queue.Queue()
        self._done = queue.Queue()
        self._workers = [threading.Thread(target=self._work, daemon=True) for _ in range(self.n_workers)]
        for t in self._workers:
            t.start()

    def _work(self):
        while True:
            job = self._jobs.get()
            if job is None:
                return
            job.time_it('started')
            try:
                job.result = self.compute(config=job.kwargs['config'], budget=job.kwargs['budget'],
                                          working_directory=job.kwargs.get('working_directory', '.'))
            except Exception as e:
                job.exception = repr(e)
                job.result = None
            job.time_it('finished')
            self._done.put(job)

    def run(self):
        if self.queue_callback is not None:
            self.queue_callback(self.n_workers)
        while True:
            job = self._done.get()
            if job is None:
                return
            if self.new_result_callback is not None:
                self.new_result_callback(job)

    def number_of_workers(self):
        return self.n_workers

    def shutdown(self, shutdown_workers=False):
        for _ in self._workers:
            self._jobs.put(None)
        self._done.put(None)

    def submit_job(self, id, **kwargs):
        job = Job(id, **kwargs)
        job.time_it('submitted')
        self._jobs.put(job)
        return job
