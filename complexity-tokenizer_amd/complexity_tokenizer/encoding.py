"""Encoding / BatchEncoding: the reference's result objects (src/encoding.rs:5-460,
src/bindings/encoding.rs:6-296), filled from the GPU's padded rows (ctok_encode_padded).

The per-encoding methods (pad, truncate, truncate_with_stride, the char/word/token lookups) are
host-side list operations, restated from src/encoding.rs with the reference's quirks kept:
  * `tokens` is not extended by the post-processor (mod.rs:378-386), so truncating between the
    token count and the id count slices past the end of `tokens` -- the reference panics there
    (Rust slice bounds), and so does this class (PanicException);
  * `pad` extends ids / type_ids / tokens / attention / special / sequence_ids, not offsets or
    word_ids (encoding.rs:87-131).

`offsets` and `word_ids` of encode_to_encoding's encodings are the reference's approximate byte
ranges (`str::find` of each pre-tokenized word, mod.rs:395-480), computed by ctok_encode_offsets
from the GPU encode's pieces.  Encodings made by Encoding.from_ids have empty offsets / word_ids,
as in the reference.  An Encoding built without them (offsets=None) raises NotImplementedError
on access rather than returning different values.
"""
from __future__ import annotations

import numpy as np

_UNKNOWN = None  # offsets / word_ids not given (see the module docstring)


def _need(v, what):
    if v is _UNKNOWN:
        raise NotImplementedError("%s were not computed for this Encoding" % what)
    return v


class Encoding:
    """src/encoding.rs:5-27 (fields) with the methods of src/bindings/encoding.rs:12-177."""

    __slots__ = ("ids", "type_ids", "tokens", "attention_mask", "special_tokens_mask", "_offsets", "_word_ids",
                 "sequence_ids", "overflowing_list")

    def __init__(self, ids, type_ids, tokens, attention_mask, special_tokens_mask, offsets, word_ids,
                 sequence_ids, overflowing=None):
        self.ids = ids
        self.type_ids = type_ids
        self.tokens = tokens
        self.attention_mask = attention_mask
        self.special_tokens_mask = special_tokens_mask
        self._offsets = offsets
        self._word_ids = word_ids
        self.sequence_ids = sequence_ids
        self.overflowing_list = overflowing if overflowing is not None else []

    # ---------------------------------------------------------------- constructors
    @staticmethod
    def from_ids(ids, tokens):
        """Encoding::from_ids (src/encoding.rs:45-58)."""
        ids = [int(i) for i in ids]
        n = len(ids)
        return Encoding(ids, [0] * n, list(tokens), [1] * n, [0] * n, [], [], [0] * n)

    # ---------------------------------------------------------------- getters
    @property
    def offsets(self):
        return list(_need(self._offsets, "offsets"))

    @property
    def word_ids(self):
        return list(_need(self._word_ids, "word_ids"))

    @property
    def overflowing(self):
        return list(self.overflowing_list)

    @property
    def n_overflowing(self):
        return len(self.overflowing_list)

    def __len__(self):
        return len(self.ids)

    def __repr__(self):
        return "Encoding(num_tokens=%d)" % len(self.ids)

    def ids_as_numpy(self):
        return np.asarray(self.ids, dtype=np.uint32)

    def attention_mask_as_numpy(self):
        return np.asarray(self.attention_mask, dtype=np.uint32)

    def type_ids_as_numpy(self):
        return np.asarray(self.type_ids, dtype=np.uint32)

    def special_tokens_mask_as_numpy(self):
        return np.asarray(self.special_tokens_mask, dtype=np.uint32)

    # ---------------------------------------------------------------- edits
    def pad(self, target_length, pad_id, pad_token, pad_left):
        """Encoding::pad (src/encoding.rs:87-131)."""
        n = len(self.ids)
        if n >= target_length:
            return
        k = target_length - n
        if pad_left:
            self.ids = [pad_id] * k + self.ids
            self.type_ids = [0] * k + self.type_ids
            self.tokens = [pad_token] * k + self.tokens
            self.attention_mask = [0] * k + self.attention_mask
            self.special_tokens_mask = [1] * k + self.special_tokens_mask
            self.sequence_ids = [None] * k + self.sequence_ids
        else:
            self.ids = self.ids + [pad_id] * k
            self.type_ids = self.type_ids + [0] * k
            self.tokens = self.tokens + [pad_token] * k
            self.attention_mask = self.attention_mask + [0] * k
            self.special_tokens_mask = self.special_tokens_mask + [1] * k
            self.sequence_ids = self.sequence_ids + [None] * k

    @staticmethod
    def _slice(v, a, b, what):
        """Rust `v[a..b]`: panics when b > len or a > b."""
        if b > len(v) or a > b:
            from . import PanicException  # (defined by the package, which imports this module)
            raise PanicException("range end index %d out of range for slice of length %d (%s)" % (b, len(v), what))
        return v[a:b]

    @staticmethod
    def _opt_slice(v, a, b, cond_len):
        """`if v.len() > cond_len { v[a..b] } else { Vec::new() }` for offsets / word_ids /
        sequence_ids, with unknown (not produced) values kept unknown."""
        if v is _UNKNOWN:
            return _UNKNOWN
        return v[a:b] if len(v) > cond_len else []

    def truncate(self, max_length):
        """Encoding::truncate (src/encoding.rs:133-181)."""
        n = len(self.ids)
        if n <= max_length:
            return
        s = self._slice
        over = Encoding(s(self.ids, max_length, n, "ids"), s(self.type_ids, max_length, len(self.type_ids), "type_ids"),
                        s(self.tokens, max_length, len(self.tokens), "tokens"),
                        s(self.attention_mask, max_length, len(self.attention_mask), "attention_mask"),
                        s(self.special_tokens_mask, max_length, len(self.special_tokens_mask), "special_tokens_mask"),
                        self._opt_slice(self._offsets, max_length, None, max_length),
                        self._opt_slice(self._word_ids, max_length, None, max_length),
                        self.sequence_ids[max_length:] if len(self.sequence_ids) > max_length else [])
        self.overflowing_list.append(over)
        self._truncate_all(max_length)

    def _truncate_all(self, m):
        self.ids = self.ids[:m]
        self.type_ids = self.type_ids[:m]
        self.tokens = self.tokens[:m]
        self.attention_mask = self.attention_mask[:m]
        self.special_tokens_mask = self.special_tokens_mask[:m]
        if self._offsets is not _UNKNOWN:
            self._offsets = self._offsets[:m]
        if self._word_ids is not _UNKNOWN:
            self._word_ids = self._word_ids[:m]
        self.sequence_ids = self.sequence_ids[:m]

    def truncate_with_stride(self, max_length, stride):
        """Encoding::truncate_with_stride (src/encoding.rs:183-231): overlapping windows.  A stride
        >= max_length never advances in the reference (an endless loop); refused here."""
        n = len(self.ids)
        if n <= max_length:
            return
        if stride >= max_length:
            raise ValueError("stride must be smaller than max_length (the reference loops forever)")
        pos = max_length
        s = self._slice
        while pos < n:
            start = max(0, pos - stride)
            end = min(start + max_length, n)

            def opt(v):
                if v is _UNKNOWN:
                    return _UNKNOWN
                return v[start:min(end, len(v))] if len(v) > start else []
            over = Encoding(s(self.ids, start, end, "ids"), s(self.type_ids, start, end, "type_ids"),
                            s(self.tokens, start, end, "tokens"), s(self.attention_mask, start, end, "attention_mask"),
                            s(self.special_tokens_mask, start, end, "special_tokens_mask"), opt(self._offsets),
                            opt(self._word_ids), opt(self.sequence_ids))
            self.overflowing_list.append(over)
            pos = end
        self._truncate_all(max_length)

    # ---------------------------------------------------------------- lookups (src/encoding.rs:263-460)
    def char_to_token(self, char_pos):
        for i, (a, b) in enumerate(self.offsets):
            if a <= char_pos < b:
                return i
        return None

    def char_to_token_with_sequence(self, char_pos, sequence_id):
        for i, (a, b) in enumerate(self.offsets):
            sid = self.sequence_ids[i] if i < len(self.sequence_ids) else None
            if sid is not None and sid == sequence_id and a <= char_pos < b:
                return i
        return None

    def token_to_chars(self, token_idx):
        off = self.offsets
        return off[token_idx] if 0 <= token_idx < len(off) else None

    def token_to_word(self, token_idx):
        w = self.word_ids
        return w[token_idx] if 0 <= token_idx < len(w) else None

    def token_to_sequence(self, token_idx):
        return self.sequence_ids[token_idx] if 0 <= token_idx < len(self.sequence_ids) else None

    def word_to_tokens(self, word_idx):
        return self.word_to_tokens_with_sequence(word_idx, 0)

    def word_to_tokens_with_sequence(self, word_idx, sequence_id=0):
        start = end = None
        for i, wid in enumerate(self.word_ids):
            if wid is None:
                continue
            sid = self.sequence_ids[i] if i < len(self.sequence_ids) else None
            if wid == word_idx and sid is not None and sid == sequence_id:
                if start is None:
                    start = i
                end = i + 1
        return (start, end) if start is not None else None

    def word_to_chars(self, word_idx):
        return self.word_to_chars_with_sequence(word_idx, 0)

    def word_to_chars_with_sequence(self, word_idx, sequence_id=0):
        rng = self.word_to_tokens_with_sequence(word_idx, sequence_id)
        if rng is None:
            return None
        cs = ce = None
        off = self.offsets
        for i in range(rng[0], rng[1]):
            if i < len(off):
                a, b = off[i]
                cs = a if cs is None or a < cs else cs
                ce = b if ce is None or b > ce else ce
        return (cs, ce) if cs is not None else None

    def word_token_indices(self, word_idx):
        return [i for i, w in enumerate(self.word_ids) if w == word_idx]

    @property
    def n_words(self):
        return len({w for w in self.word_ids if w is not None})


class BatchEncoding:
    """PyBatchEncoding (src/bindings/encoding.rs:180-296)."""

    def __init__(self, encodings, return_attention_mask=True, return_token_type_ids=True,
                 return_offsets_mapping=False, return_special_tokens_mask=False):
        self._encodings = encodings
        self.return_attention_mask = return_attention_mask
        self.return_token_type_ids = return_token_type_ids
        self.return_offsets_mapping = return_offsets_mapping
        self.return_special_tokens_mask = return_special_tokens_mask

    @property
    def input_ids(self):
        return [list(e.ids) for e in self._encodings]

    @property
    def attention_mask(self):
        return [list(e.attention_mask) for e in self._encodings] if self.return_attention_mask else []

    @property
    def token_type_ids(self):
        return [list(e.type_ids) for e in self._encodings] if self.return_token_type_ids else []

    @property
    def special_tokens_mask(self):
        return [list(e.special_tokens_mask) for e in self._encodings] if self.return_special_tokens_mask else []

    @property
    def offset_mapping(self):
        return [e.offsets for e in self._encodings] if self.return_offsets_mapping else []

    def encodings(self):
        return list(self._encodings)

    def __len__(self):
        return len(self._encodings)

    def __getitem__(self, idx):
        if not isinstance(idx, int) or idx < 0 or idx >= len(self._encodings):
            raise IndexError("Index out of range")
        return self._encodings[idx]

    def keys(self):
        k = ["input_ids"]
        if self.return_attention_mask:
            k.append("attention_mask")
        if self.return_token_type_ids:
            k.append("token_type_ids")
        if self.return_special_tokens_mask:
            k.append("special_tokens_mask")
        if self.return_offsets_mapping:
            k.append("offset_mapping")
        return k

    def to_dict(self):
        d = {"input_ids": self.input_ids}
        if self.return_attention_mask:
            d["attention_mask"] = self.attention_mask
        if self.return_token_type_ids:
            d["token_type_ids"] = self.token_type_ids
        if self.return_special_tokens_mask:
            d["special_tokens_mask"] = self.special_tokens_mask
        if self.return_offsets_mapping:
            d["offset_mapping"] = self.offset_mapping
        return d

    def input_ids_as_numpy(self):
        return [e.ids_as_numpy() for e in self._encodings]

    def attention_mask_as_numpy(self):
        return [e.attention_mask_as_numpy() for e in self._encodings]
