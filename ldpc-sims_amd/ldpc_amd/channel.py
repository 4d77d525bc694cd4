"""Device channel front ends (Python side of ldpc_awgn_llr / ldpc_ofdm_tx / ldpc_ofdm_demod).

* ``awgn_llr``   BPSK over AWGN -> LLRs (distributionally the reference's QPSK-OFDM at rate 1/2).
* ``ofdm_tx``    ``modulate_bits`` + ``transmit_symbols`` (``ofdm/ofdm_functions.py:17-35``): QPSK or
                 16-QAM (Gray, new), unitary IDFT per ``ofdm_size`` block, complex AWGN at ``snr``.
* ``ofdm_demod`` ``demodulate_signal`` (``:63-78``): unitary DFT, LLR = log P(1)/P(0).
* ``adc_quantize`` ``quantizer`` (``:37-51``) with the AGC clip of ``gen_qdata`` (``:118-128``).
* ``gen_data`` / ``gen_qdata`` — the reference's two data generators (``:109-128``), same return order.
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


def adc_quantize(rx, num_bits, clip_ratio=None, clip_value=None, want_clip=False):
    """Quantize a complex64 CUDA stream: AGC (clip = std(rx) * clip_ratio, on device) or a fixed clip."""
    if (clip_ratio is None) == (clip_value is None):
        raise ValueError("give exactly one of clip_ratio / clip_value")
    r = torch.view_as_real(rx.contiguous().view(-1)).contiguous()
    q = torch.empty_like(r)
    clip = torch.empty((1,), dtype=torch.float64, device=r.device) if want_clip else None
    _abi.check(_abi.load().ldpc_adc_quantize(r.data_ptr(), r.shape[0], int(num_bits), float(clip_ratio or 0.0),
                                             float(clip_value or 0.0), q.data_ptr(),
                                             clip.data_ptr() if clip is not None else None, _st()))
    qc = torch.view_as_complex(q)
    return (qc, clip) if want_clip else qc


def gen_data(bits, snrdb, ofdm_size=32, bits_per_symbol=2, seed=0, sym0=0):
    """``gen_data`` (``ofdm_functions.py:109-116``) from a bit stream: returns rx_signal, rx_symbols,
    rx_llrs, tx_signal (complex64 / float32 CUDA tensors)."""
    snr = 10.0 ** (snrdb / 10.0)
    rx, tx = ofdm_tx(bits, ofdm_size, bits_per_symbol, snr, seed, sym0, want_tx=True)
    llr, sym = ofdm_demod(rx, ofdm_size, bits_per_symbol, snr, want_symbols=True)
    return rx, sym, llr, tx


def gen_qdata(rx_signal, snrdb, qbits, clip_ratio, ofdm_size=32, bits_per_symbol=2):
    """``gen_qdata`` (``ofdm_functions.py:118-128``): AGC-clipped ADC, then demodulation.  Returns
    qrx_signal, qrx_symbols, qrx_llrs."""
    snr = 10.0 ** (snrdb / 10.0)
    q = adc_quantize(rx_signal, qbits, clip_ratio=clip_ratio)
    llr, sym = ofdm_demod(q, ofdm_size, bits_per_symbol, snr, want_symbols=True)
    return q, sym, llr
