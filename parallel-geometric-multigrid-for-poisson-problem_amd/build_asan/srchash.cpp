extern "C" const char *pgmg_source_hash(void) { return "asan-7cbcc07a982fff9a"; }
