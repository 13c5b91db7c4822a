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


def window_inputs(case, oracle):
    """Sources, repairs and received repair FPIDs of a window_cases.json case.  Repairs are
    recomputed with the CPU oracle: the window sender encodes its window as block number 0
    (window_framework_sender.h:215), or per repair from the block number its FPID carries when
    mixed_seeds is set; the fixture pins the oracle's encode elsewhere (encode_cases.json)."""
    k, r, L = case["k"], case["r"], case["L"]
    data = synth_bytes(k * L, case["data_seed"]).reshape(k, L)
    lens = case["src_len"]
    srcs = [data[j, : (lens[j] if lens else L)].copy() for j in range(k)]
    fpids = case["repair_fpid_raw"]
    if case["scheme"] == "xor":
        reps = [oracle.xor_encode_block(srcs)[1]]
    elif case["mixed_seeds"]:
        reps = [oracle.rlc_encode_block((fpids[i] >> 8) & 0xFFFFFF, srcs, r)[1][i] for i in range(r)]
    else:
        reps = oracle.rlc_encode_block(0, srcs, r)[1]
    return srcs, reps, fpids
