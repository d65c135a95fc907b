/*
 * k1_l9_main.c — test driver for the reference's L9 path. src/main.c defines
 * L9_data_handler (src/main.c:362-472: the L9 CSV reader, the L9 SLAM loop of
 * src/main.c:423-431 and its CSV writer) but its main() only calls the L5
 * handler (src/main.c:477-481). oracle/Makefile `k1` compiles main.c as it
 * lies with its main renamed (-Dmain=navslam_ref_l5_main) and links this
 * file, whose main calls the L9 handler instead. TEST INFRASTRUCTURE ONLY.
 */
#undef main /* the -Dmain rename is for src/main.c only */
void L9_data_handler();

int main(void)
{
    L9_data_handler();
    return 0;
}
