"""Framework logger.

Same record format as the reference logger (``distribute_log.py:10``:
``'%(asctime)s  [ %(levelname)s ]: %(message)s'``) and the same module-level
helpers ``info/warn/error/debug`` (``distribute_log.py:14-27``).  Unlike the
reference we do not call ``logging.basicConfig`` on the root logger at import
time (that hijacks the host application's logging); the ``mdtf`` logger owns a
single stream handler instead.  Rank information is prepended when running
under a multi-process job so interleaved logs stay attributable.
"""
import logging
import os
import sys

LOGGING_LEVEL = logging.INFO
FORMAT = '%(asctime)s  [ %(levelname)s ]: %(message)s'

logger = logging.getLogger("mdtf")
if not logger.handlers:
    _h = logging.StreamHandler(sys.stderr)
    _h.setFormatter(logging.Formatter(FORMAT))
    logger.addHandler(_h)
    logger.setLevel(int(os.environ.get("MDTF_LOG_LEVEL", LOGGING_LEVEL)))
    logger.propagate = False


def _prefix(message):
    rank = os.environ.get("MDTF_RANK_TAG")
    return "%s %s" % (rank, message) if rank else message


def info(message):
    logger.info(_prefix(message))


def warn(message):
    logger.warning(_prefix(message))


warning = warn


def error(message):
    logger.error(_prefix(message))


def debug(message):
    logger.debug(_prefix(message))


def set_level(level):
    logger.setLevel(level)
