# data_loader/data_loader.py -- reference-compatible entry point
# (Flink-ddd/pretraining-llm data_loader/data_loader.py:7), backed by the native
# token loader in pretraining_llm_amd/csrc/host/token_loader.cpp.
from pretraining_llm_amd.data.loader import get_batch_iterator, TokenLoader  # noqa: F401
