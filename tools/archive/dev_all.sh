#!/bin/bash
# GPU box: parity tests + bench line, rocprofv3 kernel stats, then the PMC traffic passes.
bash tools/dev_prof.sh || exit $?
bash tools/pmc.sh
