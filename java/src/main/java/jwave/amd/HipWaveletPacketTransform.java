/*
 * HipWaveletPacketTransform — WaveletPacketTransform (WaveletPacketTransform.java:73-191)
 * on libjwave_hip.so, plus a batched entry for many signals in one call.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.WaveletPacketTransform;
import jwave.transforms.wavelets.Wavelet;

public class HipWaveletPacketTransform extends WaveletPacketTransform implements HipTransform {

  private final HipNative.Taps _taps;

  public HipWaveletPacketTransform( Wavelet wavelet ) {
    super( wavelet );
    _taps = HipNative.tapsFor( wavelet );
  }

  @Override public double[ ] forward( double[ ] a, int level ) throws JWaveException {
    if( _taps == null )
      return super.forward( a, level );
    double[ ] out = new double[ a.length ];
    HipNative.check( HipNative.t1( 1, true, a, out, level, _taps ) );
    return out;
  }

  @Override public double[ ] reverse( double[ ] a, int level ) throws JWaveException {
    if( _taps == null )
      return super.reverse( a, level );
    double[ ] out = new double[ a.length ];
    HipNative.check( HipNative.t1( 1, false, a, out, level, _taps ) );
    return out;
  }

  /** WaveletTransform.decompose (WaveletTransform.java:136-145) for the packet
   *  tree in ONE native call: row p = forward(arrTime, p). */
  @Override public double[ ][ ] decompose( double[ ] arrTime ) throws JWaveException {
    if( _taps == null )
      return super.decompose( arrTime );
    int n = arrTime.length;
    int rows = 32 - Integer.numberOfLeadingZeros( Math.max( n, 1 ) );
    if( !HipNative.fitsArray( rows, n ) )  // (log2 n + 1) * n > one Java array
      return super.decompose( arrTime );
    double[ ] mat = new double[ rows * n ];
    HipNative.Taps t = _taps;
    HipNative.check( HipNative.decompose( HipNative.ctx( ), 1, arrTime, mat, t.L, t.tw, t.scale,
        t.lo, t.hi, t.loR, t.hiR ) );
    return HipNative.unpack( mat, rows, n );
  }

  @Override public HipNative.Taps taps( ) { return _taps; }

  @Override public int kind( ) { return 1; }

  // 2-D / 3-D (BasicTransform.java:361-474, 509-659) in one native call each
  @Override public double[ ][ ] forward( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( _taps == null || !HipNative.fitsArray( m.length, m.length == 0 ? 0 : m[ 0 ].length ) )
      return super.forward( m, lvlM, lvlN );
    return HipNative.run2d( 1, _taps, true, m, lvlM, lvlN );
  }

  @Override public double[ ][ ] reverse( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( _taps == null || !HipNative.fitsArray( m.length, m.length == 0 ? 0 : m[ 0 ].length ) )
      return super.reverse( m, lvlM, lvlN );
    return HipNative.run2d( 1, _taps, false, m, lvlM, lvlN );
  }

  @Override public double[ ][ ][ ] forward( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( _taps == null || !HipNative.fits3d( s ) )
      return super.forward( s, lvlP, lvlQ, lvlR );
    return HipNative.run3d( 1, _taps, true, false, s, lvlP, lvlQ, lvlR );
  }

  @Override public double[ ][ ][ ] reverse( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( _taps == null || !HipNative.fits3d( s ) )
      return super.reverse( s, lvlP, lvlQ, lvlR );
    return HipNative.run3d( 1, _taps, false, false, s, lvlP, lvlQ, lvlR );
  }

  /** Every row (one signal each, equal lengths) with the same level: one
   *  native call instead of one per signal, split over the GPUs listed in
   *  -Djwave.hip.devices when set (HipNative.batch). */
  public double[ ][ ] forwardBatch( double[ ][ ] signals, int level ) throws JWaveException {
    return batch( true, signals, level );
  }

  public double[ ][ ] reverseBatch( double[ ][ ] coeffs, int level ) throws JWaveException {
    return batch( false, coeffs, level );
  }

  private double[ ][ ] batch( boolean fwd, double[ ][ ] m, int level ) throws JWaveException {
    int rows = m.length, cols = rows == 0 ? 0 : m[ 0 ].length;
    if( _taps == null || !HipNative.fitsArray( rows, cols ) ) {
      double[ ][ ] out = new double[ rows ][ ];
      for( int i = 0; i < rows; i++ )
        out[ i ] = fwd ? super.forward( m[ i ], level ) : super.reverse( m[ i ], level );
      return out;
    }
    return HipNative.batch( 1, _taps, fwd, m, level );
  }
}
