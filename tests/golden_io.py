"""Loaders for the reference-generated fixtures in tests/golden/ (see gen_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

from oracle_py import synth_bytes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def encode_inputs(case) -> np.ndarray:
    nb, k, L = case["nblocks"], case["k"], case["L"]
    return synth_bytes(nb * k * L, case["data_seed"]).reshape(nb, k, L)


def decode_sources(case):
    """Original source symbols of a decode case (list of uint8 arrays)."""
    if "src_hex" in case:
        return [np.frombuffer(bytes.fromhex(h), np.uint8).copy() for h in case["src_hex"]]
    k, L = case["k"], case["L"]
    data = synth_bytes(k * L, case["data_seed"]).reshape(k, L)
    return [data[j].copy() for j in range(k)]
