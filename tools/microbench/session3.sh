set -u
cd /root/repo/tools/microbench
for b in pb_g1 pb_g2 pb_gnoload pb_gnoatom pb_gnone pb_g1 pb_g2; do
  echo "== $b" >> ../../gpurun_out/pb3.txt
  timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb3.txt 2>&1
  rc=$?; echo "rc=$rc" >> ../../gpurun_out/pb3.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
done
cat ../../gpurun_out/pb3.txt
