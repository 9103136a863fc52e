/*
 * HipTransform — what HipParallelTransform needs from a wrapped Hip transform:
 * the bank it sends to the GPU (null: the Java fallback) and its kind
 * (0 = FWT, 1 = WPT).
 */
package jwave.amd;

interface HipTransform {
  HipNative.Taps taps( );

  int kind( );
}
