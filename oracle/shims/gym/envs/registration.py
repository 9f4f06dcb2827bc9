import importlib

_REGISTRY = {}


def register(id, entry_point, **kwargs):
    _REGISTRY[id] = entry_point


def make(env_id):
    mod, cls = _REGISTRY[env_id].split(":")
    return getattr(importlib.import_module(mod), cls)()
