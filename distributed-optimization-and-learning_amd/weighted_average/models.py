"""Model1 / Model3 (DIST/models.py) — re-exported from the engine."""
import _engine  # noqa: F401
from dolhip.models import Model1, Model3  # noqa: F401
