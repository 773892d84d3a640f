"""klog-style verbosity on top of :mod:`logging` (reference: klog -v=N, Helm default -v=4)."""

from __future__ import annotations

import logging
import sys


def setup_logging(verbosity: int = 2, debug: bool = False):
    level = logging.DEBUG if (debug or verbosity >= 4) else (logging.INFO if verbosity >= 1 else logging.WARNING)
    logging.basicConfig(stream=sys.stderr, level=level,
                        format="%(levelname).1s%(asctime)s %(process)d %(name)s] %(message)s",
                        datefmt="%m%d %H:%M:%S")
