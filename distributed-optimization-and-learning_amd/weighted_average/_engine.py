"""Locate and import the `dolhip` engine that sits next to this directory."""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

import dolhip  # noqa: E402,F401
