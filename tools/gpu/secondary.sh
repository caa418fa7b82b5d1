set -o pipefail
B="timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline"
$B > gpurun_out/sec_headline.json 2> gpurun_out/sec_headline.err && \
$B --solver GMRES > gpurun_out/sec_pseudo.json 2> gpurun_out/sec_pseudo.err && \
$B --prec right > gpurun_out/sec_jacobi.json 2> gpurun_out/sec_jacobi.err && \
$B --solver "FLEXIBLE GMRES" --prec right --sweeps 2 > gpurun_out/sec_flex.json 2> gpurun_out/sec_flex.err && \
$B --matrix Brick3D --prec right > gpurun_out/sec_brick.json 2> gpurun_out/sec_brick.err
