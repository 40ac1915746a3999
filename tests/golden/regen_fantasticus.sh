#!/bin/sh
# Regenerates the consensus goldens on the bundled F.antasticus sample from the reference Perl engine.
# Runs only in the build container (needs /root/reference); outputs are committed.
set -e
cd "$(dirname "$0")"
python3 make_fantasticus_cases.py fantasticus/cns_cases.txt
PERL_HASH_SEED=0 PERL_PERTURB_KEYS=0 perl gen_cns_golden.pl fantasticus/cns_cases.txt > fantasticus/cns_expected.txt
