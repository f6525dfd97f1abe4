#!/bin/bash
# GS parity tests + 256^3 GS trace per team size + 512^3 GS run.
set -u
TAG=${TAG:-gs_all} TEAMS="${TEAMS:-64 16}" bash scripts/r04/gs_check.sh || exit 1
TAG=${TAG:-gs_all}_512 TEAM=${TEAM512:-64} bash scripts/r04/gs512.sh
