"""Algorithm registry.

Same API as the reference (`method/algorithm_factory.py:6-79`):
`CentralizedAlgorithmFactory.register_algorithm(algorithm_name, client_cls, server_cls,
client_endpoint_cls=None, server_endpoint_cls=None, algorithm_cls=None)`, `has_algorithm`,
`create_client(algorithm_name, kwargs, endpoint_kwargs, extra_kwargs, extra_endpoint_kwargs)`,
`create_server(...)` (instantiates `algorithm_cls()` and injects it as `algorithm=`).
"""

from __future__ import annotations

from typing import Callable

from ..topology import ClientEndpoint, ServerEndpoint


class CentralizedAlgorithmFactory:
    config: dict[str, dict] = {}

    @classmethod
    def register_algorithm(cls, algorithm_name: str, client_cls: Callable, server_cls: Callable,
                           client_endpoint_cls: Callable | None = None,
                           server_endpoint_cls: Callable | None = None,
                           algorithm_cls: Callable | None = None) -> None:
        assert algorithm_name not in cls.config, algorithm_name
        cls.config[algorithm_name] = {
            "client_cls": client_cls,
            "server_cls": server_cls,
            "client_endpoint_cls": client_endpoint_cls or ClientEndpoint,
            "server_endpoint_cls": server_endpoint_cls or ServerEndpoint,
        }
        if algorithm_cls is not None:
            cls.config[algorithm_name]["algorithm_cls"] = algorithm_cls

    @classmethod
    def has_algorithm(cls, algorithm_name: str) -> bool:
        return algorithm_name in cls.config

    @classmethod
    def create_client(cls, algorithm_name: str, kwargs: dict, endpoint_kwargs: dict,
                      extra_kwargs: dict | None = None, extra_endpoint_kwargs: dict | None = None):
        cfg = cls.config[algorithm_name]
        endpoint = cfg["client_endpoint_cls"](**(endpoint_kwargs | (extra_endpoint_kwargs or {})))
        return cfg["client_cls"](endpoint=endpoint, **(kwargs | (extra_kwargs or {})))

    @classmethod
    def create_server(cls, algorithm_name: str, kwargs: dict, endpoint_kwargs: dict,
                      extra_kwargs: dict | None = None, extra_endpoint_kwargs: dict | None = None):
        cfg = cls.config[algorithm_name]
        extra_kwargs = dict(extra_kwargs or {})
        endpoint = cfg["server_endpoint_cls"](**(endpoint_kwargs | (extra_endpoint_kwargs or {})))
        if "algorithm_cls" in cfg:
            assert "algorithm" not in extra_kwargs
            extra_kwargs["algorithm"] = cfg["algorithm_cls"]()
        return cfg["server_cls"](endpoint=endpoint, **(kwargs | extra_kwargs))
