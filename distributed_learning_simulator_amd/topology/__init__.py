from .endpoints import (ClientEndpoint, NNADQClientEndpoint, NNADQServerEndpoint,
                        QuantClientEndpoint, QuantServerEndpoint, ServerEndpoint,
                        StochasticQuantClientEndpoint, StochasticQuantServerEndpoint)

__all__ = [
    "ClientEndpoint", "ServerEndpoint", "QuantClientEndpoint", "QuantServerEndpoint",
    "StochasticQuantClientEndpoint", "StochasticQuantServerEndpoint",
    "NNADQClientEndpoint", "NNADQServerEndpoint",
]
