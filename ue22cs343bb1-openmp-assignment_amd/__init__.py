"""MI355X-native batched DASH directory-coherence simulator (libdash).

The directory name is not a Python identifier; load it with
`importlib` (see __graft_entry__.load_package) or put this directory on
sys.path and `import dash`.
"""
from .dash import *  # noqa: F401,F403
