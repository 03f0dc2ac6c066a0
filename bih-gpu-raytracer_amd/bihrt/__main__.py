"""python -m bihrt: the presentation-free frame loop (bihrt/app.py)."""
import sys

from .app import main

sys.exit(main())
