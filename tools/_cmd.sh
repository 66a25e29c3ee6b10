set -u
bash tools/gpu_session.sh r03b tests || exit $?
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r03b_ko base=default scan=$V/libzfft_scan.so corr=$V/libzfft_corr.so lo=$V/libzfft_lo.so ld=$V/libzfft_ld.so st=$V/libzfft_st.so fwd=$V/libzfft_fwd.so
