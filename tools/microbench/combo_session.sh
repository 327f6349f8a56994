cd tools/microbench && timeout -k 5 120 ./wpat > ../../gpurun_out/wpat.txt 2>&1
cd /root/repo && tools/microbench/run_rb.sh rb_old rb_new rb_spread rb_nostore
cd tools/microbench && for b in pb_new pb_nodma pb_new pb_nodma; do echo "== $b" >> ../../gpurun_out/pb.txt; timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb.txt 2>&1 || echo "$b rc=$?" >> ../../gpurun_out/pb.txt; done
cat ../../gpurun_out/pb.txt
