set -o pipefail
for cfg in "1024 256 8 256 3 1 1" "1024 128 16 128 3 1 1" "1024 512 4 512 3 1 1" "1024 1024 8 256 1 1 0" "1024 256 8 1024 1 1 0" "1024 512 16 128 1 1 0" "1024 128 16 512 1 1 0" "1024 256 32 64 1 1 0"; do
  echo "== $cfg"; timeout -k 10 60 python -u tools/wgrad_probe.py $cfg || exit 1
done
