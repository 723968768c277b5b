"""Device-map planner and checkpoint loading helpers re-exported under `utils` (parity: reference
utils/modeling.py big-model helpers). Implementation lives in `_big_modeling_impl` and `hooks`."""

_IMPL_NAMES = (
    "infer_auto_device_map",
    "get_balanced_memory",
    "get_max_memory",
    "load_checkpoint_in_model",
    "set_module_tensor_to_device",
    "get_max_layer_size",
    "check_device_map",
    "clean_device_map",
    "load_state_dict",
    "calculate_maximum_sizes",
    "find_tied_parameters",
    "retie_parameters",
)
_HOOK_NAMES = ("align_module_device", "has_offloaded_params")


def __getattr__(name):
    if name in _IMPL_NAMES:
        from .. import _big_modeling_impl

        return getattr(_big_modeling_impl, name)
    if name in _HOOK_NAMES:
        from .. import _big_modeling_impl, hooks

        return getattr(_big_modeling_impl, name, None) or getattr(hooks, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


def infer_auto_device_map(*args, **kwargs):
    from .._big_modeling_impl import infer_auto_device_map as f

    return f(*args, **kwargs)


def load_checkpoint_in_model(*args, **kwargs):
    from .._big_modeling_impl import load_checkpoint_in_model as f

    return f(*args, **kwargs)
