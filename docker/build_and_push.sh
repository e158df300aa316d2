#!/bin/bash
# Build the framework image from the repo root and push it to REGISTRY (default: local tag only).
set -euxo pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-homebrewnlp-mtf-amd:latest}
docker build -f docker/Dockerfile -t "$TAG" .
if [ -n "${REGISTRY:-}" ]; then
  docker tag "$TAG" "$REGISTRY/$TAG"
  docker push "$REGISTRY/$TAG"
fi
