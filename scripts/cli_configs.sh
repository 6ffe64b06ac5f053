#!/bin/bash
# Device join time of the phjoin CLI on the reference's partition counts (10M x 200M, device-generated).
set -o pipefail
cd "$(dirname "$0")/.."
for args in "--join radix-partitioning -p 32" "--join radix-partitioning -p 1024" "--join radix-partitioning --radix-bits 8,8 --hash murmur3" "--join radix-partitioning -p 65536" "--join no-partitioning" "--join radix-partitioning --radix-bits 8,8 --hash murmur3 --skew 1.25"; do
  timeout -k 10 120 ./partitionedhashjoin_amd/phjoin $args --generate device --log error -u us -f /tmp/cli_out.txt > /dev/null 2>/tmp/cli_err.txt || { echo "FAILED: $args"; tail -3 /tmp/cli_err.txt; exit 1; }
  echo "$args :: $(tr -d '\n ' < /tmp/cli_out.txt)"
done
