#!/bin/bash
# Build the committed (HEAD) sources as montecarlopathtracer_amd/lib/$1 (default
# libmcpt_base.so) for an A/B against the working tree's libmcpt.so.
set -e
NAME=${1:-libmcpt_base.so}
git stash push -q -- montecarlopathtracer_amd/csrc include
trap 'git stash pop -q' EXIT
MCPT_LIB_NAME=$NAME python montecarlopathtracer_amd/_build.py --force > /dev/null 2>&1
