"""Multi-process (gloo, world_size 2, CPU) test of the N > 1 path: byte-balanced doc sharding,
per-rank encode, gather with token-offset rebasing.  The per-rank encoder here is the C oracle
(the GPU encoder is exercised by the -m gpu tests); the sharding/rebase logic is the product's
(complexity_tokenizer.parallel), identical for both."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tok_path, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "complexity-tokenizer_amd")]
    import torch.distributed as dist

    from complexity_tokenizer.parallel import encode_sharded
    from datagen import corpus
    from oracle import ref_c

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rc = ref_c.RefC.from_file(tok_path)
    text, off = corpus.corpus_c2(20_000, seed=31)
    ids, toff, _ = encode_sharded(lambda t, o: rc.encode_packed(t, o, threads=2), text, off, rank, world)
    if rank == 0:
        np.savez(out_path, ids=ids, toff=toff)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single(gpt2_path, tmp_path):
    from datagen import corpus
    from oracle import ref_c

    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), gpt2_path, out), nprocs=2, join=True)
    got = np.load(out)
    text, off = corpus.corpus_c2(20_000, seed=31)
    ids, toff = ref_c.RefC.from_file(gpt2_path).encode_packed(text, off)
    assert np.array_equal(got["toff"], toff)
    assert np.array_equal(got["ids"], ids)
