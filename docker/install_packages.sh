#!/bin/bash
# System + Python dependencies of the framework image (docker/Dockerfile). Strict mode: any failure stops the build.
set -euo pipefail
export DEBIAN_FRONTEND=noninteractive
apt-get update
apt-get install -y --no-install-recommends ffmpeg zlib1g-dev git make
python3 -m pip install --no-cache-dir -r /tmp/requirements.txt
apt-get clean
rm -rf /var/lib/apt/lists/*
