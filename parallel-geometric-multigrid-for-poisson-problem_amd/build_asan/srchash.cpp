extern "C" const char *pgmg_source_hash(void) { return "asan-456c43c436f0f475"; }
