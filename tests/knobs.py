"""Contexts with switches: libndfl.so reads its NDFL_* switches once, when a context is created
(ndfl_common.hpp Knobs), so a test that needs a decoder or encoder path a switch selects creates its
own context with the switch set."""
import os


def context(device=0, **env):
    """ndfl.Context(device) created with the given NDFL_* environment (restored afterwards)."""
    import ndfl
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = str(v)
    try:
        return ndfl.Context(device)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
