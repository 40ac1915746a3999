#!/bin/sh
# ChimeraToSeqFilter.pl drop-in (proovread calls it by this name): chimera annotations -> SeqFilter --substr.
HERE=$(cd "$(dirname "$0")/.." && pwd)
PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" exec python3 -m proovread_amd.chimera_filter "$@"
