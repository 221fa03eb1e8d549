"""`python -m shellac_amd ...` runs the proxy CLI (same flags as `shellac`)."""
import sys

from .server.proxy import main

sys.exit(main())
