set -u
for sz in "1048576 1472" "524288 2944" "262144 5888" "131072 11776" "65536 23552" "23552 65536"; do
  set -- $sz
  echo "== $1 x $2"
  timeout -k 10 120 python tools/ab.py cyclone_amd/libcyaes.so --rounds 6 --payloads $1 --payload-bytes $2 || exit 1
done
