"""python -m guacamole_amd <command> [args] — the Command registry (Guacamole.scala:37-44)
restricted to the two callers on the accelerated path."""
import sys

from .commands import main

sys.exit(main())
