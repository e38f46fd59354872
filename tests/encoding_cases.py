"""Tokenizer variants and texts for the padded-encode / Encoding tests:
the GPT-2-shaped fixture with special added tokens and each post-processor the reference parses
(src/huggingface/parsing.rs:193-253)."""
import copy

from tests import edge_cases

SPECIALS = ["[CLS]", "[SEP]", "[PAD]", "<s>", "</s>", "<|bos|>"]


def with_post_processor(base_obj, kind):
    obj = copy.deepcopy(base_obj)
    nid = max(obj["model"]["vocab"].values()) + 1
    added = list(obj.get("added_tokens", []))
    for k, tok in enumerate(SPECIALS):
        added.append({"id": nid + k, "content": tok, "single_word": False, "lstrip": False, "rstrip": False,
                      "normalized": False, "special": True})
    obj["added_tokens"] = added
    if kind == "template":
        obj["post_processor"] = {"type": "TemplateProcessing",
                                 "single": [{"SpecialToken": {"id": "<|bos|>", "type_id": 0}},
                                            {"Sequence": {"id": "A", "type_id": 0}},
                                            {"SpecialToken": {"id": "[SEP]", "type_id": 0}}],
                                 "pair": [{"Sequence": {"id": "A", "type_id": 0}},
                                          {"SpecialToken": {"id": "[SEP]", "type_id": 0}},
                                          {"Sequence": {"id": "B", "type_id": 1}}]}
    elif kind == "template_twice":  # $A twice and an unknown special token name (skipped)
        obj["post_processor"] = {"type": "TemplateProcessing",
                                 "single": [{"Sequence": {"id": "A", "type_id": 0}},
                                            {"SpecialToken": {"id": "[CLS]", "type_id": 0}},
                                            {"SpecialToken": {"id": "<unknown>", "type_id": 0}},
                                            {"Sequence": {"id": "A", "type_id": 0}}]}
    elif kind == "template_no_a":  # no $A: the reference panics unless the specials outnumber the ids
        obj["post_processor"] = {"type": "TemplateProcessing",
                                 "single": [{"SpecialToken": {"id": "[CLS]", "type_id": 0}}]}
    elif kind == "bert":
        obj["post_processor"] = {"type": "BertProcessing", "sep": ["[SEP]", 0], "cls": ["[CLS]", 0]}
    elif kind == "roberta":
        obj["post_processor"] = {"type": "RobertaProcessing", "sep": ["</s>", 0], "cls": ["<s>", 0]}
    elif kind == "sequence":  # parsed as None by the reference
        obj["post_processor"] = {"type": "Sequence", "processors": []}
    else:
        obj["post_processor"] = None
    return obj


def texts():
    out = ["hello world", "", "a", " [CLS] inside [SEP] text", "<s>roberta</s>", "multi\nline\ttext  here",
           "numbers 12345 and punctuation!!!", "x" * 70, "the " * 40]
    out += [e for e in edge_cases.EDGE if e][:30]
    return out
