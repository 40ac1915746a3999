#!/bin/sh
# Regenerates the trim-window / quality-run goldens from the reference Fastq::Seq module.
# Runs only in the build container (needs /root/reference); outputs are committed.
set -e
cd "$(dirname "$0")"
python3 make_seqfilter_cases.py seqfilter_cases.txt
PERL_HASH_SEED=0 PERL_PERTURB_KEYS=0 perl gen_seqfilter_golden.pl seqfilter_cases.txt > seqfilter_expected.txt
