"""Model families used by the pipeline: the language identifier (hashed character 1-4-gram
int16 logit table, csrc/common/langid.h) and the TokenCounter tokenizer wrapper."""
