# GPU box: host issue cost of the config B step (tools/host_cost_b.py) with the in-tree Python
# package and with tools/old_host/{_native,engine}.py in a copy of the tree.  Usage: bash tools/ab_host.sh OUT
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/host_ab}; mkdir -p $O
rm -rf /tmp/oldrepo && mkdir -p /tmp/oldrepo && cp -r bench.py __graft_entry__.py oracle tools movierecommender-tf-trt_amd /tmp/oldrepo/ && cp tools/old_host/_native.py tools/old_host/engine.py /tmp/oldrepo/movierecommender-tf-trt_amd/movierec/
for r in 1 2; do
  timeout -k 10 120 python tools/host_cost_b.py > $O/new_$r.txt 2>&1; head -1 $O/new_$r.txt | sed "s/^/new $r: /"
  (cd /tmp/oldrepo && timeout -k 10 120 python tools/host_cost_b.py) > $O/old_$r.txt 2>&1; head -1 $O/old_$r.txt | sed "s/^/old $r: /"
done
