set -e
for v in 1 3; do
  for b in FULL NOLOAD NOMFMA; do
    echo "variant=$v $b: $(LLP_GEMM_VARIANT=$v timeout -k 5 60 tools/bin/ablate_$b)"
    echo "variant=$v $b small-A: $(LLP_GEMM_VARIANT=$v timeout -k 5 60 tools/bin/ablate_$b 747214 small)"
  done
done
