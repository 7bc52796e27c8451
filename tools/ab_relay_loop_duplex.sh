# tools/ab_relay_loop_duplex.sh -- relay_loop (both relay ends through the
# batcher) with large chunks, the batcher's two directions side by side
# (default) against one after the other (CYAES_DUPLEX=0), alternating.
set -e
R=build/relay_loop
ARGS="--threads 8 --pipes 4 --chunks 8 --size rand:65280 --recv-copy 0 --seconds 3 --depth 2"
for i in 1 2 3 4 5; do
  echo "== round $i duplex"; timeout -k 10 60 $R $ARGS
  echo "== round $i two launches (CYAES_DUPLEX=0)"; CYAES_DUPLEX=0 timeout -k 10 60 $R $ARGS
done
