#!/bin/sh
# Regenerates the full-size consensus goldens (bwa-sr-1 and bwa-sr-finish cases, 10 kb reads)
# from the reference Perl engine.  Runs only in the build container (needs /root/reference);
# the gzipped outputs are committed.
set -e
cd "$(dirname "$0")"
T=$(mktemp -d)
python3 make_scale_cases.py "$T"
for k in bwa_sr1 finish; do
    PERL_HASH_SEED=0 PERL_PERTURB_KEYS=0 perl gen_cns_golden.pl "$T/${k}_cases.txt" > "$T/${k}_expected.txt"
    gzip -9 -n -c "$T/${k}_cases.txt" > scale/${k}_cases.txt.gz
    gzip -9 -n -c "$T/${k}_expected.txt" > scale/${k}_expected.txt.gz
done
rm -rf "$T"
