#!/bin/sh
# Regenerates the consensus golden fixtures from the reference Perl engine.
# Runs only in the build container (needs /root/reference); outputs are committed.
set -e
cd "$(dirname "$0")"
python3 make_cns_cases.py cns_cases.txt 48
PERL_HASH_SEED=0 PERL_PERTURB_KEYS=0 perl gen_cns_golden.pl cns_cases.txt > cns_expected.txt
