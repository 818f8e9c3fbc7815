#!/usr/bin/env bash
# Convert rocprofv3 rocpd databases merged into gpurun_out/ into markdown
# kernel summaries under profiles/ (tracked). Usage: rocprof_to_profiles.sh <tag>
set -euo pipefail
cd "$(dirname "$0")/.."
tag=${1:-latest}
mkdir -p profiles
for db in gpurun_out/${tag}_rocprof_*/*.db gpurun_out/rocprof_*/*.db; do
  [ -f "$db" ] || continue
  name=$(basename "$(dirname "$db")")
  tmp=$(mktemp -d)
  /opt/rocm/bin/rocpd2summary -i "$db" -f md -d "$tmp" -o "$name" >/dev/null 2>&1 || true
  for f in "$tmp"/*.md; do
    [ -f "$f" ] && cp "$f" "profiles/${tag}_$(basename "$f")"
  done
  rm -rf "$tmp"
done
ls profiles
