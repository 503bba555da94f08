#!/bin/bash
# kernel trace of the headline steps on the current library
set -o pipefail
cd "$(dirname "$0")/../.."
bash profiles/collect.sh r05al 20 trace-only
