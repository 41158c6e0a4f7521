"""Top-level module name replicat imports (replicat/utils/adapters.py:10: `import
_replicat_adapters`).  Re-exports the MI355X drop-in from replicat_amd; put the repository
root on sys.path (or install this file next to replicat) to switch replicat over."""
from replicat_amd._replicat_adapters import _gclmulchunker  # noqa: F401

__all__ = ['_gclmulchunker']
