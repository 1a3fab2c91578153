"""coldforce_amd -- MI355X-native WebSocket frame codec for coldforce.

The product is ``libcfws.so`` (built from ``csrc/`` by the top-level
Makefile): a C ABI that keeps coldforce's ``co_ws_frame_*`` symbols
(``include/cfws_co_ws_frame.h``) and adds a batch codec over device arenas
(``include/cfws.h``). ``cfws`` is its ctypes binding; ``workloads`` builds
the BASELINE.json frame batches.
"""
from . import cfws  # noqa: F401

__all__ = ["cfws"]
