"""Device-map planner and checkpoint loading helpers (see big_modeling.py)."""


def infer_auto_device_map(*args, **kwargs):
    from .._big_modeling_impl import infer_auto_device_map as f

    return f(*args, **kwargs)


def load_checkpoint_in_model(*args, **kwargs):
    from .._big_modeling_impl import load_checkpoint_in_model as f

    return f(*args, **kwargs)
