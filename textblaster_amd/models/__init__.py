"""Model families used by the pipeline: the language identifier (fastText-style char n-gram
embedding bag + bf16 MFMA linear head) and the TokenCounter tokenizer wrapper."""
