"""ldpc_amd — MI355X-native LDPC belief-propagation decoding (gfx950 HIP kernels behind a C ABI).

Drop-in for the decode path of realjwin/ldpc-sims (pytorch/bp + ofdm_functions.decode_bits).
"""
from . import _abi, codes
from .api import Decoder, decode, decode_bits, decoder, get_decoder
from .codes import Encoder, Graph, QCCode, get_code, peg_64_32, qc_expand, wifi_code

_abi.load()  # fail loudly at import if the HIP library is missing: there is no CPU fallback

__all__ = ["Decoder", "decode", "decode_bits", "decoder", "get_decoder", "BeliefPropagation", "codes",
           "Encoder", "Graph", "QCCode", "get_code", "peg_64_32", "qc_expand", "wifi_code"]


def __getattr__(name):
    if name == "BeliefPropagation":
        from . import api
        return api.BeliefPropagation
    raise AttributeError(name)
