set -e
for args in "129 100 512" "129 100 1024" "129 100 1536" "129 100 2048" "129 80 1024" "129 80 2048"; do timeout -k 5 60 tools/bin/bulk_probe $args 5 | grep -v checksum; done
