"""Synthetic codewords on device (test/bench data generation; not on the decode path).

Dense-H codes: parity = info @ Gp (mod 2) with the systematic parity map from codes.Encoder.
IRA codes kept sparse (codes.SparseCode, e.g. the DVB-S2-shaped code): check sums of the information
bits by index_add, then the staircase accumulator p_c = p_{c-1} xor s_c as a cumulative sum mod 2.
"""
from __future__ import annotations

import numpy as np

from .codes import Encoder, IRAEncoder, SparseCode


class DeviceEncoder:
    def __init__(self, H, device):
        import torch
        self.torch = torch
        self.device = device
        if isinstance(H, SparseCode):
            e = IRAEncoder(H)
            self.k, self.m = e.k, e.m
            self.chk = torch.from_numpy(e._chk.astype(np.int64)).to(device)
            self.col = torch.from_numpy(e._col.astype(np.int64)).to(device)
            self.Gp = None
        else:
            e = Encoder(H)
            self.k, self.m = e.k, e.m
            self.Gp = torch.from_numpy(e.generator_parity().astype(np.float32)).to(device)

    def encode(self, info):
        """info: uint8 (B, k) on device -> codewords uint8 (B, n)."""
        torch = self.torch
        if self.Gp is not None:
            par = torch.remainder(info.float() @ self.Gp, 2.0).to(torch.uint8)
        else:
            s = torch.zeros((info.shape[0], self.m), dtype=torch.int32, device=info.device)
            s.index_add_(1, self.chk, info[:, self.col].to(torch.int32))
            par = (torch.cumsum(s, dim=1) & 1).to(torch.uint8)
        return torch.cat([info.to(torch.uint8), par], dim=1).contiguous()
