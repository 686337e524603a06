# Round 5: tools/microbench/bin_chunk, one process per pattern (each under its own limit)
O=gpurun_out/${TAG:-r5mb}
mkdir -p $O
for m in seq direct atomics pre xcdpre chunkx chunk; do
  timeout -k 5 40 ./tools/microbench/bin_chunk 100000000 $m >> $O/bin_chunk.txt 2>&1
  rc=$?
  echo "$m rc=$rc" >> $O/bin_chunk.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
