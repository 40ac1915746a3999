// Host-only statistics build of the seeding core (tools/seed_stats.sh): seed.cpp compiled with
// -DPR_SEED_STATS, so seed_core.h's SC_STAT counters (occurrence lookups, occurrences visited,
// chain searches, merges, new chains, shifted list elements, ...) add into pr_seed_stat_g.
#include <cstring>

unsigned long long pr_seed_stat_g[24];

int pr_set_error(int code, const char *) { return code; }
extern "C" void pr_seed_stat_get(unsigned long long *out) { std::memcpy(out, pr_seed_stat_g, sizeof(pr_seed_stat_g)); }
extern "C" void pr_seed_stat_reset() { std::memset(pr_seed_stat_g, 0, sizeof(pr_seed_stat_g)); }
