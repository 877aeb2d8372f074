"""Builds two small stand-in ``tokenizer.json`` files for the TokenCounter tests.

The reference's token-counter tests download ``bert-base-uncased`` and ``gpt2`` from the Hub
(reference token_counter.rs:52-148). There is no network here, so these fixtures reproduce the
*pipeline structure* of those tokenizers (BERT: lowercase + BertPreTokenizer + WordPiece +
``[CLS] $A [SEP]``; GPT-2: ByteLevel BPE, no special tokens) over a tiny vocabulary. They are not
the real vocabularies: only the reference tests' sentences are pinned (11 / 9 / 2 tokens).

    python tools/make_test_tokenizers.py tests/fixtures/tokenizers
"""
import os
import sys

from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

CORPUS = ["Hello, world! This is a test.", "hello world this is a test", "Another test sentence, with words."] * 50


def bert(out_dir):
    vocab = {t: i for i, t in enumerate(
        ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "hello", "world", "this", "is", "a", "test", ",", "!", ".",
         "another", "sentence", "with", "words", "##s"])}
    tok = Tokenizer(models.WordPiece(vocab=vocab, unk_token="[UNK]"))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
        special_tokens=[("[CLS]", vocab["[CLS]"]), ("[SEP]", vocab["[SEP]"])])
    tok.decoder = decoders.WordPiece()
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))


def gpt2(out_dir):
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=400, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  special_tokens=["<|endoftext|>"])
    tok.train_from_iterator(CORPUS, trainer)
    tok.post_processor = processors.ByteLevel(trim_offsets=False)
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))


if __name__ == "__main__":
    base = sys.argv[1] if len(sys.argv) > 1 else "tests/fixtures/tokenizers"
    bert(os.path.join(base, "bert-base-uncased"))
    gpt2(os.path.join(base, "gpt2"))
    for name in ("bert-base-uncased", "gpt2"):
        t = Tokenizer.from_file(os.path.join(base, name, "tokenizer.json"))
        print(name, len(t.encode("Hello, world! This is a test.").tokens), len(t.encode("").tokens))
