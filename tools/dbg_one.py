"""Encode a few texts with the GPT-2-shaped fixture (debugging aid for a single call)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "complexity-tokenizer_amd"))
from datagen.build_tokenizers import fixture_path  # noqa: E402
from complexity_tokenizer import Tokenizer  # noqa: E402

path = fixture_path(sys.argv[1] if len(sys.argv) > 1 else "gpt2_50k", tempfile.mkdtemp())
tok = Tokenizer.from_file(path)
tok.device = 0
texts = [sys.argv[2] if len(sys.argv) > 2 else "x" * 70]
print("encoding", [len(t) for t in texts], flush=True)
print(tok.encode_batch(texts)[0][:20], flush=True)
