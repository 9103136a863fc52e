/*
 * HipFastWaveletTransform — FastWaveletTransform whose per-level loops
 * (FastWaveletTransform.java:71-153) and the 2-D/3-D loops inherited from
 * BasicTransform (BasicTransform.java:361-474, 509-659) run as single calls
 * into libjwave_hip.so.  Drop-in: new Transform( new HipFastWaveletTransform( w ) ).
 * Wavelets the native path does not reproduce fall back to the Java code.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.FastWaveletTransform;
import jwave.transforms.wavelets.Wavelet;

public class HipFastWaveletTransform extends FastWaveletTransform implements HipTransform {

  protected final HipNative.Taps _taps;
  protected final int _kind;

  public HipFastWaveletTransform( Wavelet wavelet ) { this( wavelet, 0 ); }

  protected HipFastWaveletTransform( Wavelet wavelet, int kind ) {
    super( wavelet );
    _taps = HipNative.tapsFor( wavelet );
    _kind = kind;
  }

  protected double[ ] superForward( double[ ] a, int level ) throws JWaveException {
    return super.forward( a, level );
  }

  protected double[ ] superReverse( double[ ] a, int level ) throws JWaveException {
    return super.reverse( a, level );
  }

  @Override public double[ ] forward( double[ ] arrTime, int level ) throws JWaveException {
    if( _taps == null )
      return superForward( arrTime, level );
    double[ ] out = new double[ arrTime.length ];
    HipNative.check( HipNative.t1( _kind, true, arrTime, out, level, _taps ) );
    return out;
  }

  @Override public double[ ] reverse( double[ ] arrHilb, int level ) throws JWaveException {
    if( _taps == null )
      return superReverse( arrHilb, level );
    double[ ] out = new double[ arrHilb.length ];
    HipNative.check( HipNative.t1( _kind, false, arrHilb, out, level, _taps ) );
    return out;
  }

  /**
   * WaveletTransform.decompose (WaveletTransform.java:136-145) in ONE native
   * call: row p = forward(arrTime, p) for p = 0..log2 n (jwv_decompose_f64).
   * recompose(m, level) is the inherited reverse(m[level], level) (:173-182).
   */
  @Override public double[ ][ ] decompose( double[ ] arrTime ) throws JWaveException {
    if( _taps == null )
      return super.decompose( arrTime );
    int n = arrTime.length;
    int rows = 32 - Integer.numberOfLeadingZeros( Math.max( n, 1 ) );  // log2 n + 1 for 2^p
    if( !HipNative.fitsArray( rows, n ) )  // (log2 n + 1) * n > one Java array
      return super.decompose( arrTime );
    double[ ] mat = new double[ rows * n ];
    HipNative.Taps t = _taps;
    HipNative.check( HipNative.decompose( HipNative.ctx( ), _kind, arrTime, mat, t.L, t.tw,
        t.scale, t.lo, t.hi, t.loR, t.hiR ) );
    return HipNative.unpack( mat, rows, n );
  }

  /** Every row (one signal each, equal lengths) with the same level: one
   *  native call, split over the GPUs of -Djwave.hip.devices when set. */
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
        out[ i ] = fwd ? forward( m[ i ], level ) : reverse( m[ i ], level );
      return out;
    }
    return HipNative.batch( _kind, _taps, fwd, m, level );
  }

  /** The bank this transform sends to the GPU, or null (Java fallback). */
  @Override public HipNative.Taps taps( ) { return _taps; }

  @Override public int kind( ) { return _kind; }

  @Override public double[ ][ ] forward( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( _taps == null || !HipNative.fitsArray( m.length, m.length == 0 ? 0 : m[ 0 ].length ) )
      return super.forward( m, lvlM, lvlN );
    return HipNative.run2d( _kind, _taps, true, m, lvlM, lvlN );
  }

  @Override public double[ ][ ] reverse( double[ ][ ] m, int lvlM, int lvlN )
      throws JWaveException {
    if( _taps == null || !HipNative.fitsArray( m.length, m.length == 0 ? 0 : m[ 0 ].length ) )
      return super.reverse( m, lvlM, lvlN );
    return HipNative.run2d( _kind, _taps, false, m, lvlM, lvlN );
  }

  @Override public double[ ][ ][ ] forward( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( _taps == null || !HipNative.fits3d( s ) )
      return super.forward( s, lvlP, lvlQ, lvlR );
    return HipNative.run3d( _kind, _taps, true, false, s, lvlP, lvlQ, lvlR );
  }

  @Override public double[ ][ ][ ] reverse( double[ ][ ][ ] s, int lvlP, int lvlQ, int lvlR )
      throws JWaveException {
    if( _taps == null || !HipNative.fits3d( s ) )
      return super.reverse( s, lvlP, lvlQ, lvlR );
    return HipNative.run3d( _kind, _taps, false, false, s, lvlP, lvlQ, lvlR );
  }
}
