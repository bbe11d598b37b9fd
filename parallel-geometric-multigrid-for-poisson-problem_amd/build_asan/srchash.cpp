extern "C" const char *pgmg_source_hash(void) { return "asan-e2100b8b7f5440bc"; }
