#!/bin/bash
# r4 quick session: k-NN GPU tests, then A/B probe + bench of the query
# passes and the k_knnw stamps
TAG=${1:-r4s}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
PYTEST_K="${PYTEST_K:-knn or pair or smoke}" bash scripts/r4_knn_ab.sh "$TAG" || exit $?
bash scripts/r4_stamps.sh "$TAG/st"
