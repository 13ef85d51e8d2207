"""a5x -- MI355X-native backend for hashcat -a 5 table-attack candidate expansion.

Drop-in for the expansion hot path of ``A113L/hashcat_a5_table_generator``
(``main.go:164-440``): the Go CLI, the ``.table`` format and the ``cand\\n`` output
stay as they are; the per-word engines run as gfx950 HIP kernels behind the C ABI
of ``include/a5x.h`` (``_build/liba5x.so``).
"""
from ._lib import A5xError, LIB_PATH
from .engine import (ALGO_MD5, ALGO_NTLM, DeviceBuffer, MODE_DEFAULT, MODE_REVERSE, MODE_SUBALL, MODE_SUBALL_REVERSE, Context, decode_hex_notation,
                     format_plain, generate, mode_of, pack_words, partition, process_word, process_word_reverse,
                     process_word_substitute_all, process_word_substitute_all_reverse, read_substitution_table,
                     split_words)

__all__ = [
    "A5xError", "LIB_PATH", "ALGO_MD5", "ALGO_NTLM", "Context", "DeviceBuffer", "MODE_DEFAULT", "MODE_REVERSE", "MODE_SUBALL", "MODE_SUBALL_REVERSE",
    "decode_hex_notation", "format_plain", "generate", "mode_of", "pack_words", "partition", "process_word",
    "process_word_reverse", "process_word_substitute_all", "process_word_substitute_all_reverse",
    "read_substitution_table", "split_words",
]
