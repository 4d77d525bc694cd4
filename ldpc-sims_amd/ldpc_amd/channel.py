"""Device channel front ends (Python side of ldpc_awgn_llr / ldpc_ofdm_tx / ldpc_ofdm_demod).

* ``awgn_llr``   BPSK over AWGN -> LLRs (distributionally the reference's QPSK-OFDM at rate 1/2).
* ``ofdm_tx``    ``modulate_bits`` + ``transmit_symbols`` (``ofdm/ofdm_functions.py:17-35``): QPSK or
                 16-QAM (Gray, new), unitary IDFT per ``ofdm_size`` block, complex AWGN at ``snr``.
* ``ofdm_demod`` ``demodulate_signal`` (``:63-78``): unitary DFT, LLR = log P(1)/P(0).
Torch GPU tensors in/out (current stream).
"""
from __future__ import annotations

import torch

from . import _abi


def _st():
    return torch.cuda.current_stream().cuda_stream


def awgn_llr(codewords, sigma, seed=0, b0=0):
    B, n = codewords.shape
    out = torch.empty((B, n), dtype=torch.float32, device=codewords.device)
    _abi.check(_abi.load().ldpc_awgn_llr(codewords.data_ptr(), out.data_ptr(), B, n, float(sigma), int(seed), int(b0), _st()))
    return out


def ofdm_tx(bits, ofdm_size=32, bits_per_symbol=2, snr=1.0, seed=0, sym0=0, want_tx=False):
    """bits: uint8 CUDA tensor of nsym * bits_per_symbol bits (a stream).  Returns complex64 rx (and tx)."""
    bits = bits.contiguous().view(-1)
    nsym = bits.numel() // bits_per_symbol
    rx = torch.empty((nsym, 2), dtype=torch.float32, device=bits.device)
    tx = torch.empty((nsym, 2), dtype=torch.float32, device=bits.device) if want_tx else None
    _abi.check(_abi.load().ldpc_ofdm_tx(bits.data_ptr(), nsym, ofdm_size, bits_per_symbol, float(snr), int(seed),
                                        int(sym0), rx.data_ptr(), tx.data_ptr() if tx is not None else None, _st()))
    rxc = torch.view_as_complex(rx)
    return (rxc, torch.view_as_complex(tx)) if want_tx else rxc


def ofdm_demod(rx, ofdm_size=32, bits_per_symbol=2, snr=1.0, want_symbols=False):
    """rx: complex64 CUDA tensor (stream of samples).  Returns float32 LLRs (nsym * bits_per_symbol)."""
    r = torch.view_as_real(rx.contiguous().view(-1)).contiguous()
    nsym = r.shape[0]
    llr = torch.empty((nsym * bits_per_symbol,), dtype=torch.float32, device=r.device)
    sym = torch.empty((nsym, 2), dtype=torch.float32, device=r.device) if want_symbols else None
    _abi.check(_abi.load().ldpc_ofdm_demod(r.data_ptr(), nsym, ofdm_size, bits_per_symbol, float(snr), llr.data_ptr(),
                                           sym.data_ptr() if sym is not None else None, _st()))
    return (llr, torch.view_as_complex(sym)) if want_symbols else llr
