"""Layout helpers, synthetic inputs, verification metrics, reporting."""
from . import inputs, layout, metrics  # noqa: F401
