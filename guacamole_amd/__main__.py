"""python -m guacamole_amd <command> [args] — the Command registry (Guacamole.scala:37-44)
restricted to the two callers on the accelerated path."""
import os
import sys

from . import _early

_early.start(sys.argv[1:])  # the GPU context opens on a host thread while the imports below run

from . import bamdev  # noqa: E402
from .commands import main  # noqa: E402

bamdev.DEFER_RELEASE = True  # this process ends after the command: the loaders' buffers go with it
rc = main()
# The output is written and closed: end the process here rather than tear the interpreter down
# (collecting the resident read sets' device buffers one hipFree at a time and the HIP runtime's
# exit add ~0.1 s to a single pass); the device loaders' release threads finish first.
from .bamdev import join_release_threads  # noqa: E402

join_release_threads()
sys.stdout.flush()
sys.stderr.flush()
os._exit(rc)
