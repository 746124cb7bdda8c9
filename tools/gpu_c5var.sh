# C5 ring-chain instance: one level per wave on 8 waves (production) against two levels
# per wave on 4 (var/kw2*), timed and digest-checked, twice.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/c5var}
mkdir -p $D
for rep in 1 2; do
  timeout -k 10 500 python3 -u tools/c5_variants.py mpi-model_amd/libmpimodel_hip.so var/kw1/libmpimodel_hip.so \
      var/kw2/libmpimodel_hip.so var/kw2b4/libmpimodel_hip.so var/kw2u1/libmpimodel_hip.so >> $D/c5var.log 2>&1 \
      || { tail -20 $D/c5var.log; exit 1; }
done
cat $D/c5var.log
