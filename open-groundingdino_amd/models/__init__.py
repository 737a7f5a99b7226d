"""Reference-compatible model package: ``models.registry.MODULE_BUILD_FUNCS``
and ``models.GroundingDINO.build_groundingdino`` (reference models/__init__.py,
models/registry.py), so the reference's main.py/engines import this package
unchanged once ``open-groundingdino_amd/`` is on sys.path."""
from .GroundingDINO import build_groundingdino  # noqa: F401


def build_model(args):
    from .registry import MODULE_BUILD_FUNCS
    return MODULE_BUILD_FUNCS.get(args.modelname)(args)
