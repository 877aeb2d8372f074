#!/bin/bash
# Quick developer build of the host extension (the package build lives in textblaster_amd/native.py)
set -e
cd "$(dirname "$0")/.."
python -c "from textblaster_amd import native; native.build_host(verbose=True)"
