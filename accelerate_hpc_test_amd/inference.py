"""Pipeline-parallel inference (`prepare_pippy`). Implementation: parallel/pipeline.py."""


def prepare_pippy(*args, **kwargs):
    from .parallel.pipeline import prepare_pippy as f

    return f(*args, **kwargs)
