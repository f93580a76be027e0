#!/bin/bash
set -o pipefail
O=gpurun_out/r6rm; mkdir -p $O
PYTHONPATH=. timeout -k 10 120 python -u bench/dbg/rm_forms_diag.py 100 > $O/rm_forms_100.jsonl 2> $O/rm_forms.err &&
PYTHONPATH=. timeout -k 10 120 python -u bench/dbg/rm_forms_diag.py 400 > $O/rm_forms_400.jsonl 2>> $O/rm_forms.err
