# dense_mv with random values: the footprint knee, and alternating the stream direction per pass
for sc in 0.5 0.75 1.0 1.25 1.5 2.0; do for alt in 0 1; do echo "alt $alt"; timeout -k 5 60 scripts/micro/bin/dense_mv $sc 0 0 1 $alt || exit 1; done; done > gpurun_out/dense_knee_rand.txt 2>&1
cat gpurun_out/dense_knee_rand.txt
