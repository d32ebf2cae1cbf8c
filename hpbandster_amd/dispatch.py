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
