"""base_config_generator -- the drop-in contract (reference: hpbandster/config_generators/base.py:6-69).

``get_config(budget) -> (config_dict, info_dict)`` and ``new_result(job)``; ``new_result`` logs the
job through the optional result logger and warns about failed jobs, exactly like the reference.
"""

import logging

from ..utils import json_result_logger


class base_config_generator(object):
    def __init__(self, directory=None, result_logger=json_result_logger, overwrite=False, logger=None):
        if directory is not None:
            self.result_logger = result_logger(directory, overwrite=overwrite)
        else:
            self.result_logger = None
        self.logger = logging.getLogger('hpbandster') if logger is None else logger

    def get_config(self, budget):
        raise NotImplementedError('This function needs to be overwritten in %s.' % (self.__class__.__name__))

    def new_result(self, job):
        if self.result_logger is not None:
            self.result_logger(job)
        if job.exception is not None:
            self.logger.warning("job {} failed with exception\n{}".format(job.id, job.exception))
