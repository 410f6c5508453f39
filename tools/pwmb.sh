for sh in "32 32 24000" "16 32 24000" "64 64 12000" "32 64 12000" "128 128 3000" "64 128 3000" "256 256 600" "128 256 600"; do
  for pw in 0 1; do echo "ENCX_PW=$pw $sh"; ENCX_PW=$pw timeout -k 5 30 tools/mb/conv_mb $sh 1 1 2>&1 | grep -E "encx|conv|B 32" | head -4; done
done
