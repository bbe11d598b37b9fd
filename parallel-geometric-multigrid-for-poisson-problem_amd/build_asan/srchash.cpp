extern "C" const char *pgmg_source_hash(void) { return "asan-f800e860cd4a5ed5"; }
