extern "C" const char *pgmg_source_hash(void) { return "asan-6ce97a80c44b809e"; }
