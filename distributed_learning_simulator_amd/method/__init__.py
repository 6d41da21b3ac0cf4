"""Importing this package registers every method (reference `method/__init__.py:1-9`)."""

from . import fed_avg  # noqa: F401
from .algorithm_factory import CentralizedAlgorithmFactory

for _m in ("fed_dropout_avg", "fed_paq", "fed_obd", "shapley_value", "sign_sgd", "smafd",
           "fed_gnn", "fed_gcn", "fed_aas"):
    try:
        __import__(f"{__name__}.{_m}")
    except ModuleNotFoundError as e:  # method package not present yet
        if not str(e).endswith(f"{_m}'"):
            raise

__all__ = ["CentralizedAlgorithmFactory"]
